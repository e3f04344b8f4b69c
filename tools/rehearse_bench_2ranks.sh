#!/bin/bash
# Rehearse bench.py's multi-rank ZeRO-3 path (deferred reduce-scatter, params retained across
# micro-steps, reuse-distance keeps) with 2 ranks sharing ONE MI355X over gloo (RCCL needs one GPU
# per rank; the real N-GPU runs are the driver's). Reduced layer count => not a metric run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 WORLD_SIZE=2 LOCAL_RANK=0 SXE_DIST_BACKEND=gloo
pids=()
for r in 0 1; do
  RANK=$r timeout -k 10 600 python -u bench.py --gpus 2 --layers ${LAYERS:-4} --steps 2 --warmup 1 \
    > gpurun_out/rehearse_rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
tail -2 gpurun_out/rehearse_rank0.log
exit $rc
