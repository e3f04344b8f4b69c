#!/bin/bash
# Round-6 batch 22: static priority for waves 4-7 of the 8-wave attention kernels (SXE_FA_PRIO) --
# flash tests with it on, kernel A/B, headline A/B.
set -o pipefail
O=gpurun_out/r06/batch22
mkdir -p $O
SXE_FA_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
S="8,2048,2048,32,8,128,1;4,2048,2048,32,8,128,1;1,32768,32768,4,1,128,1;1,32768,32768,32,8,128,1;4,2048,2048,32,8,128,0"
for t in 0 1 0 1; do
  SXE_FA_PRIO=$t timeout -k 10 300 python tools/attn_bench.py --shapes "$S" --no-sdpa > $O/attn_prio$t.log 2>&1 \
      || { tail -30 $O/attn_prio$t.log; exit 1; }
  echo "prio=$t"; python -c "
import json
for l in open('$O/attn_prio$t.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['B'], d['Sq'], d['H'], d['Hk'], d['D'], d['causal'], 'fwd', d['fwd_ms'], d['fwd_TF'], 'fb', d['fwdbwd_ms'], d['fwdbwd_TF'])"
done
