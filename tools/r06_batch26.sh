#!/bin/bash
# Round-6 batch 26: SP-32k step profile with the per-layer checkpoint policy (13 of 32 MLPs).
set -o pipefail
O=gpurun_out/r06/batch26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --config llama8b-sp32k --steps 2 --warmup 2 \
    > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
f=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/step_profile.py $f --top 30 > $O/sp32k_step.md && head -24 $O/sp32k_step.md | cut -c1-150
rm -rf $O/prof
