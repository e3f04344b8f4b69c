#!/bin/bash
# Round-6 batch 13: dual-layout LM-head gradient + fused QKV-projection/attention node -- GPU tests,
# then the headline A/B (both on = default vs both off), interleaved.
set -o pipefail
O=gpurun_out/r06/batch13
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dual_layout_gpu.py tests/test_kernels_gpu.py tests/test_flash_attn_gpu.py -x -q \
    --timeout 120 --timeout-method thread -k "dual or xent or cross_entropy or qkv or packed" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in on off on off; do
  if [ $t = on ]; then e="SXE_XENT_DUAL=1 SXE_QKV_TN=1"; else e="SXE_XENT_DUAL=0 SXE_QKV_TN=0"; fi
  env $e timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/ab_$t.log 2>&1 || { tail -30 $O/ab_$t.log; exit 1; }
  echo "headline $t $(grep '^{' $O/ab_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
done
