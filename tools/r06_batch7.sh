#!/bin/bash
# Round-6 measurement batch 7: software-pipelined flash forward (SXE_FA_FWD_PIPE) -- the flash GPU
# tests, then an interleaved A/B of the forward on the training shapes.
set -o pipefail
O=gpurun_out/r06/batch7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 300 --timeout-method thread \
    > $O/flash_tests.log 2>&1 || { tail -40 $O/flash_tests.log; exit 1; }
tail -1 $O/flash_tests.log
SH="4,2048,2048,32,8,128,1;4,2048,2048,32,8,128,0;4,2048,2048,32,8,64,1;1,32768,32768,4,1,128,1;1,8192,8192,32,8,128,1"
for rep in 1 2; do
  for p in 0 1; do
    SXE_FA_FWD_PIPE=$p timeout -k 10 300 python tools/attn_bench.py --shapes "$SH" --no-sdpa > $O/ab_pipe${p}_$rep.log 2>&1 \
        || { tail -20 $O/ab_pipe${p}_$rep.log; exit 1; }
    echo "pipe=$p rep=$rep"; grep '^{' $O/ab_pipe${p}_$rep.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['B'],d['Sq'],d['H'],d['Hk'],d['D'],d['causal'],'fwd',d['fwd_ms'],d['fwd_TF'],'fb',d['fwdbwd_ms'],d['fwdbwd_TF'])"
  done
done
