#!/bin/bash
# One GPU-box session: kernel tests, smoke, short bench. Each GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup ${BENCH_WARMUP:-1} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log; tail -3 gpurun_out/smoke.log 2>/dev/null; tail -5 gpurun_out/bench.log 2>/dev/null
exit $rc
