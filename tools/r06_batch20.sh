#!/bin/bash
# Round-6 batch 20: Mixtral-EP step profile (last full step) of the round-6 tree.
set -o pipefail
O=gpurun_out/r06/batch20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --config mixtral-ep --steps 2 --warmup 2 \
    > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
f=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/step_profile.py $f --top 40 > $O/mixtral_step.md && head -44 $O/mixtral_step.md | cut -c1-160
rm -rf $O/prof
