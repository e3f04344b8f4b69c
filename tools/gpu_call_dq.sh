#!/bin/bash
# decode GEMM kernels (skinny bf16 / fp8 / dequant): GPU tests, then the decode bench over weight
# formats, then an A/B of the same modes with the previous launch choices (SXE_DQ_U=1: one dequant
# step per round; SXE_SG_LEGACY_NW=1: no occupancy clamp on the wave count)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_skinny_gemm_gpu.py tests/test_mx_gemm_gpu.py tests/test_hf_inference_gpu.py tests/test_grouped_gemm_q_gpu.py tests/test_decode_graphs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dq_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dq_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/decode_bench.py --batches 1,16 --modes ${DQ_MODES:-graphs+mxfp8,graphs+mxfp6,graphs+mxfp4,graphs+int8,graphs+int4} > gpurun_out/decode_q.log 2>&1; rc=$?; grep mode gpurun_out/decode_q.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$DQ_AB_MODES" ]; then
  SXE_DQ_U=1 SXE_SG_LEGACY_NW=1 timeout -k 10 500 python -u tools/decode_bench.py --batches 1,16 --modes $DQ_AB_MODES > gpurun_out/decode_q_legacy.log 2>&1; rc=$?
  echo "--- legacy launch choices"; grep mode gpurun_out/decode_q_legacy.log; exit $rc
fi
