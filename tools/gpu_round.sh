#!/bin/bash
# Full GPU validation round: kernel/model tests, smoke, bench, rocprofv3 kernel stats of one step.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup ${BENCH_WARMUP:-1} > gpurun_out/bench.log 2>&1 \
 && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
      python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
find gpurun_out/prof -name "*kernel_trace.csv" -size +60M -delete
exit $rc
