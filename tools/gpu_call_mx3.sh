#!/bin/bash
# MX GEMM + FX-compile GPU tests, then the MX bench (each step time-limited).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_mx_gemm_gpu.py tests/test_compile_fx.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mx_tests.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python tools/mx_gemm_bench.py > gpurun_out/mx_bench.log 2>&1; rc2=$?; cat gpurun_out/mx_bench.log; exit $rc2
fi
exit $rc
