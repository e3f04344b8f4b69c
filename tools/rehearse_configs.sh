#!/bin/bash
# Every bench.py config on the one-GPU box:
#  (1) N=1 at the config's own size (what one MI355X holds: bench.py cuts mixtral / 70B by default);
#  (2) a 2-rank rehearsal of the multi-rank path with both ranks sharing GPU 0 over gloo (RCCL needs
#      one GPU per rank; the real N-GPU runs are the driver's), layer counts cut to fit two ranks.
# Each run has its own time limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rehearse
export PYTHONPATH=$PWD
one() {  # config, extra args
  local c=$1; shift
  timeout -k 10 ${T1:-600} python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 "$@" \
    > gpurun_out/rehearse/${c}_n1.log 2>&1
  local rc=$?; tail -1 gpurun_out/rehearse/${c}_n1.log; return $rc
}
two() {  # config, port, extra args
  local c=$1 port=$2; shift 2
  local pids=() rc=0
  for r in 0 1; do
    MASTER_ADDR=127.0.0.1 MASTER_PORT=$port WORLD_SIZE=2 RANK=$r LOCAL_RANK=0 SXE_DIST_BACKEND=gloo \
      timeout -k 10 ${T2:-600} python -u bench.py --gpus 2 --config $c --steps 2 --warmup 1 "$@" \
      > gpurun_out/rehearse/${c}_n2_rank$r.log 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  tail -1 gpurun_out/rehearse/${c}_n2_rank0.log; return $rc
}
for c in ${CONFIGS:-llama8b-z3-default mixtral-ep llama70b-infinity llama8b-sp32k}; do
  one $c || exit $?
done
[ -n "$NO_TWO" ] && exit 0
two llama8b-z3 29701 --layers 4 && two llama8b-z3-default 29703 --layers 4 && two mixtral-ep 29705 --layers 2 \
  && two llama70b-infinity 29707 --layers 2 && two llama8b-sp32k 29709 --layers 4
