#!/bin/bash
# Round-6 batch 19: SP-32k at the auto layer count (13) vs 15; batch-1 decode kernel profile.
set -o pipefail
O=gpurun_out/r06/batch19
mkdir -p $O
for t in auto n15 auto; do
  if [ $t = n15 ]; then a="--ac-layers 15"; else a=""; fi
  timeout -k 10 400 python bench.py --config llama8b-sp32k --steps 4 --warmup 2 $a > $O/sp32k_$t.log 2>&1 || { tail -30 $O/sp32k_$t.log; exit 1; }
  echo "sp32k $t $(grep '^{' $O/sp32k_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["config"].get("activation_checkpointing"))')"
done
timeout -k 10 300 python tools/decode_bench.py --batches 1 --modes graphs --steps 64 > $O/decode.log 2>&1 || { tail -30 $O/decode.log; exit 1; }
grep -v "^\[" $O/decode.log | tail -3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/decode_prof -o run -- python tools/decode_bench.py --batches 1 --modes graphs --steps 64 > $O/decode_prof.log 2>&1 || { tail -30 $O/decode_prof.log; exit 1; }
f=$(ls $O/decode_prof/*kernel_stats.csv $O/decode_prof/*/*kernel_stats.csv 2>/dev/null | head -1)
cp $f $O/decode_kernel_stats.csv
rm -rf $O/decode_prof
head -25 $O/decode_kernel_stats.csv | cut -c1-200
