#!/bin/bash
# Round-6 batch 9: two-segment wgrad kernel tests; Mixtral-EP deferral A/B (cat-free); headline check
# that the single-segment wgrad kernel did not regress.
set -o pipefail
O=gpurun_out/r06/batch9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" \
    > $O/wgrad_tests.log 2>&1 || { tail -30 $O/wgrad_tests.log; exit 1; }
tail -1 $O/wgrad_tests.log
for rep in 1 2; do
  for d in 1 0; do
    SXE_MOE_DEFER_WGRAD=$d timeout -k 10 300 python bench.py --config mixtral-ep --steps 4 --warmup 2 > $O/mixtral_defer${d}_$rep.log 2>&1 \
        || { tail -30 $O/mixtral_defer${d}_$rep.log; exit 1; }
    echo "defer=$d rep=$rep $(grep '^{' $O/mixtral_defer${d}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("peak_mem_gb"))')"
  done
done
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/headline.log 2>&1 || { tail -30 $O/headline.log; exit 1; }
echo "headline $(grep '^{' $O/headline.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
