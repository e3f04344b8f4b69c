#!/bin/bash
# Bounded TunableOp search over the Llama-3-8B GEMM shapes; each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 ${TUNE_LIMIT:-900} python3 tools/tune_gemms.py gpurun_out/tunableop_llama3_8b.csv ${TUNE_ARGS} > gpurun_out/tune.log 2>&1
rc=$?
grep -v alive gpurun_out/tune.log | tail -45
exit $rc
