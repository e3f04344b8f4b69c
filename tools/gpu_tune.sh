#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python3 tools/tune_gemms.py gpurun_out/tunableop_llama3_8b.csv > gpurun_out/tune.log 2>&1; rc=$?
tail -5 gpurun_out/tune.log; ls -la gpurun_out/*.csv; head -5 gpurun_out/tunableop_llama3_8b*.csv
[ $rc -eq 0 ] || exit $rc
f=$(ls gpurun_out/tunableop_llama3_8b*.csv | head -1)
SXE_TUNABLEOP_FILE=$f timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_tuned.log 2>&1; tail -1 gpurun_out/bench_tuned.log
timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_untuned.log 2>&1; tail -1 gpurun_out/bench_untuned.log
