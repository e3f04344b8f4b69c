#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attnprof
timeout -k 10 300 python3 tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attnprof -o attn -- python3 tools/attn_bench.py 1 > gpurun_out/attn_prof.log 2>&1
rc=$?
cat gpurun_out/attn_bench.log
f=$(find gpurun_out/attnprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-150 "$f" | head -15
exit $rc
