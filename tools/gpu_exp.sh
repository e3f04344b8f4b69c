#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_exp.py > gpurun_out/gemm_exp.log 2>&1; cat gpurun_out/gemm_exp.log
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_tuned.log 2>&1; tail -2 gpurun_out/bench_tuned.log
ls -la gpurun_out/*.csv
