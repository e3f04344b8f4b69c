#!/bin/bash
# Round-6 batch 21: 70B-Infinity (no checkpointing now) with the asynchronous host tier vs sync, interleaved.
set -o pipefail
O=gpurun_out/r06/batch21
mkdir -p $O
for t in async sync async sync; do
  if [ $t = async ]; then e="SXE_OFFLOAD_ASYNC=1"; else e="SXE_OFFLOAD_ASYNC=0"; fi
  env $e timeout -k 10 500 python bench.py --config llama70b-infinity --steps 4 --warmup 2 > $O/inf_$t.log 2>&1 \
      || { tail -30 $O/inf_$t.log; exit 1; }
  echo "infinity $t $(grep '^{' $O/inf_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
