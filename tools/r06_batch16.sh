#!/bin/bash
# Round-6 batch 16: skewed 8-wave flash forward (SXE_FA_FWD_SKEW) -- oracle tests, kernel A/B at the
# headline / SP-32k / D64 shapes, then the headline A/B.
set -o pipefail
O=gpurun_out/r06/batch16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "skew or fwd_variants" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
S="8,2048,2048,32,8,128,1;4,2048,2048,32,8,128,1;1,32768,32768,4,1,128,1;4,2048,2048,32,8,64,1;4,2048,2048,32,8,128,0"
for t in 0 1 0 1; do
  SXE_FA_FWD_SKEW=$t timeout -k 10 300 python tools/attn_bench.py --shapes "$S" --no-sdpa > $O/attn_skew$t.log 2>&1 \
      || { tail -30 $O/attn_skew$t.log; exit 1; }
  echo "skew=$t"; python -c "
import json
for l in open('$O/attn_skew$t.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['B'], d['Sq'], d['H'], d['Hk'], d['D'], d['causal'], 'fwd', d['fwd_ms'], d['fwd_TF'], 'fb', d['fwdbwd_ms'], d['fwdbwd_TF'])"
done
for t in 1 0 1 0; do
  SXE_FA_FWD_SKEW=$t timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/headline_skew$t.log 2>&1 || { tail -30 $O/headline_skew$t.log; exit 1; }
  echo "headline skew=$t $(grep '^{' $O/headline_skew$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
