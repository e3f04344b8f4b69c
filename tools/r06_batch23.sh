#!/bin/bash
# Round-6 batch 23: DeepCompile vs eager on the round-6 tree (stages 1-3), then per-arm kernel
# profiles of ZeRO-2 (last full step each).
set -o pipefail
O=gpurun_out/r06/batch23
mkdir -p $O
timeout -k 10 600 python tools/compile_bench.py --stages 1,2,3 > $O/compile_bench.log 2>&1 || { tail -30 $O/compile_bench.log; exit 1; }
grep '^{' $O/compile_bench.log | cut -c1-160
export TMPDIR=/tmp
for arm in eager compiled; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$arm -o run -- python tools/compile_bench.py --stages 2 --only $arm \
      > $O/prof_$arm.log 2>&1 || { tail -30 $O/prof_$arm.log; exit 1; }
  f=$(ls $O/prof_$arm/*kernel_trace.csv $O/prof_$arm/*/*kernel_trace.csv 2>/dev/null | head -1)
  python tools/step_profile.py $f --top 30 > $O/step_$arm.md && head -3 $O/step_$arm.md
  rm -rf $O/prof_$arm
done
