#!/bin/bash
# decode o_proj with the KV-split merge as its prologue: GPU tests, then the decode bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest tests/test_skinny_gemm_gpu.py tests/test_paged_attention_gpu.py tests/test_decode_graphs_gpu.py tests/test_hf_inference_gpu.py tests/test_inference_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/merge_tests.log 2>&1
rc=$?; tail -3 gpurun_out/merge_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/decode_bench.py --batches 1,16,64 --modes ${MODES:-graphs,graphs+fp8,graphs+fp4} > gpurun_out/decode_merge.log 2>&1; rc=$?; grep mode gpurun_out/decode_merge.log; exit $rc
