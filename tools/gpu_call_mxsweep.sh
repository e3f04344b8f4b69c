#!/bin/bash
# MX GEMM: LDS-DMA variant correctness (forced tile 6), then a tile sweep (each step time-limited).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
SXE_MX_TILE=${MX_TEST_TILE:-6} timeout -k 10 300 python -u -m pytest tests/test_mx_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mx_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/mx_sweep.log
for v in ${MX_TILES:-1 3 6}; do
  SXE_MX_TILE=$v timeout -k 10 120 python tools/mx_gemm_bench.py --quick >> gpurun_out/mx_sweep.log 2>&1 || exit $?
done
cat gpurun_out/mx_sweep.log
