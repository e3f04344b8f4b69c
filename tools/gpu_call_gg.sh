#!/bin/bash
# grouped GEMM: GPU tests with the 256x256 LDS-DMA tile forced, then the bench. Each step time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
SXE_GG_TILE=256 timeout -k 10 300 python -u -m pytest tests/test_grouped_gemm.py tests/test_moe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/grouped_gemm_bench.py > gpurun_out/gg_bench.log 2>&1; rc=$?; grep "\[" gpurun_out/gg_bench.log; exit $rc
