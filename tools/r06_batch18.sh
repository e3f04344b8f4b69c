#!/bin/bash
# Round-6 batch 18: Llama-3-70B ZeRO-Infinity with the HBM-budget checkpoint policy (auto: none at
# 10 layers) vs full-layer checkpointing, interleaved; SP-32k at the auto layer count vs 21;
# then the final per-config evidence run.
set -o pipefail
O=gpurun_out/r06/batch18
mkdir -p $O
for t in auto full auto full; do
  timeout -k 10 500 python bench.py --config llama70b-infinity --steps 4 --warmup 2 --ac-policy $t > $O/inf_$t.log 2>&1 \
      || { tail -30 $O/inf_$t.log; exit 1; }
  echo "infinity $t $(grep '^{' $O/inf_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["config"].get("activation_checkpointing"))')"
done
for t in auto n21 auto n21; do
  if [ $t = n21 ]; then a="--ac-layers 21"; else a=""; fi
  timeout -k 10 400 python bench.py --config llama8b-sp32k --steps 4 --warmup 2 $a > $O/sp32k_$t.log 2>&1 || { tail -30 $O/sp32k_$t.log; exit 1; }
  echo "sp32k $t $(grep '^{' $O/sp32k_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["config"].get("activation_checkpointing"))')"
done
bash tools/r06_final.sh
