#!/bin/bash
# Probe + MX / FX-compile GPU tests (each step time-limited; stops on a crash or timeout).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
ok_or_fail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
bash tools/gpu_call_probe.sh > /dev/null 2>&1; rc=$?; ok_or_fail $rc || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_mx_gemm_gpu.py tests/test_compile_fx.py tests/test_sparse_attention.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mx_tests.log; exit $rc
