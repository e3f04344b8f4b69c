#!/bin/bash
# MX / FPxWeight GPU tests and the MX bench (each step time-limited).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_mx_gemm_gpu.py tests/test_fp_quantizer.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mx_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mx_gemm_bench.py > gpurun_out/mx_bench.log 2>&1; rc=$?; cat gpurun_out/mx_bench.log; exit $rc
