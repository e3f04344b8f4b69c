#!/bin/bash
# Round-6 batch 8: block-sparse softmax tests, Mixtral-EP with / without deferred expert weight
# gradients (interleaved), Mixtral step attribution, then the whole GPU suite.
set -o pipefail
O=gpurun_out/r06/batch8
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_sparse_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/sparse_tests.log 2>&1 || { tail -30 $O/sparse_tests.log; exit 1; }
tail -1 $O/sparse_tests.log
for rep in 1 2; do
  for d in 1 0; do
    SXE_MOE_DEFER_WGRAD=$d timeout -k 10 300 python bench.py --config mixtral-ep --steps 4 --warmup 2 > $O/mixtral_defer${d}_$rep.log 2>&1 \
        || { tail -30 $O/mixtral_defer${d}_$rep.log; exit 1; }
    echo "defer=$d rep=$rep $(grep '^{' $O/mixtral_defer${d}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("tflops_per_gpu"), d.get("peak_mem_gb"))')"
  done
done
SXE_BENCH_TORCH_PROFILE=$O/mixtral_attrib timeout -k 10 300 python bench.py --config mixtral-ep --steps 2 --warmup 2 > $O/mixtral_attrib.log 2>&1 \
    || { tail -30 $O/mixtral_attrib.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 \
    || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
