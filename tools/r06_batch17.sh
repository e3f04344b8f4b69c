#!/bin/bash
# Round-6 batch 17: smoke + the whole GPU suite; SP-32k with the partial MLP-checkpoint policy
# (auto: the first N layers only) vs MLP recompute in all 32 layers, interleaved.
set -o pipefail
bash tools/r06_suite.sh || exit 1
O=gpurun_out/r06/batch17
mkdir -p $O
for t in auto all auto all; do
  if [ $t = all ]; then a="--ac-layers 32"; else a=""; fi
  timeout -k 10 400 python bench.py --config llama8b-sp32k --steps 4 --warmup 2 $a > $O/sp32k_$t.log 2>&1 || { tail -30 $O/sp32k_$t.log; exit 1; }
  echo "sp32k $t $(grep '^{' $O/sp32k_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["config"].get("activation_checkpointing"))')"
done
