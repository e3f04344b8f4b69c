#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (counters are collected in separate runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
  python3 bench.py --steps ${BENCH_STEPS:-1} --warmup ${BENCH_WARMUP:-1} ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1
rc=$?
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -40 "$f" | cut -c1-220
tail -3 gpurun_out/prof_bench.log
# keep the big per-dispatch trace out of the merge-back budget
find gpurun_out/prof -name "*kernel_trace.csv" -size +50M -delete
exit $rc
