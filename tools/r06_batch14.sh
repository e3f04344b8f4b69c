#!/bin/bash
# Round-6 batch 14: headline step profile after the dual-layout changes; SP-32k and Mixtral-EP A/B of
# the dual-layout LM-head gradient + fused QKV node (both on = default vs both off).
set -o pipefail
O=gpurun_out/r06/batch14
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 2 --warmup 2 \
    > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
f=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/step_profile.py $f --top 40 > $O/headline_step.md && head -5 $O/headline_step.md
rm -rf $O/prof
for cfg in llama8b-sp32k mixtral-ep; do
  for t in on off on off; do
    if [ $t = on ]; then e="SXE_XENT_DUAL=1 SXE_QKV_TN=1"; else e="SXE_XENT_DUAL=0 SXE_QKV_TN=0"; fi
    env $e timeout -k 10 400 python bench.py --config $cfg --steps 4 --warmup 2 > $O/${cfg}_$t.log 2>&1 || { tail -30 $O/${cfg}_$t.log; exit 1; }
    echo "$cfg $t $(grep '^{' $O/${cfg}_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
  done
done
