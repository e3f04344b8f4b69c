#!/bin/bash
# Round-6 batch 15: GPU tests of the dual-layout paths + held bf16 weight gradients (acc2_bf16_);
# headline A/B of the held gradients; headline step profile; SP-32k / Mixtral-EP A/B of all three
# round-6 step changes (default vs SXE_XENT_DUAL=0 SXE_QKV_TN=0 SXE_WGRAD_STASH=0).
set -o pipefail
O=gpurun_out/r06/batch15
mkdir -p $O
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_dual_layout_gpu.py -x -v --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in on off on off; do
  if [ $t = on ]; then e="SXE_WGRAD_STASH=1"; else e="SXE_WGRAD_STASH=0"; fi
  env $e timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/stash_$t.log 2>&1 || { tail -30 $O/stash_$t.log; exit 1; }
  echo "headline stash $t $(grep '^{' $O/stash_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 2 --warmup 2 \
    > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
f=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/step_profile.py $f --top 40 > $O/headline_step.md && head -4 $O/headline_step.md
rm -rf $O/prof
for cfg in llama8b-sp32k mixtral-ep; do
  for t in on off; do
    if [ $t = on ]; then e="SXE_XENT_DUAL=1"; else e="SXE_XENT_DUAL=0 SXE_QKV_TN=0 SXE_WGRAD_STASH=0"; fi
    env $e timeout -k 10 400 python bench.py --config $cfg --steps 4 --warmup 2 > $O/${cfg}_$t.log 2>&1 || { tail -30 $O/${cfg}_$t.log; exit 1; }
    echo "$cfg $t $(grep '^{' $O/${cfg}_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
  done
done
