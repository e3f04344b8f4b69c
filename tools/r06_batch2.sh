#!/bin/bash
# Round-6 measurement batch 2: llama70b-infinity (10 layers on 1 GPU) host tier, synchronous vs the
# asynchronous tier under its copy schedules (windowed D2H issue, kernel-driven H2D).
set -o pipefail
O=gpurun_out/r06/infinity
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" SXE_OFFLOAD_TRACE=1 timeout -k 10 400 python bench.py --config llama70b-infinity --steps 4 --warmup 2 \
      > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'])"
}
run sync SXE_OFFLOAD_ASYNC=0
run async_w2_k1 SXE_OFFLOAD_ASYNC=1 SXE_OFFLOAD_ASYNC_WINDOW=2 SXE_OFFLOAD_H2D_KERNEL=1
run async_w0_k1 SXE_OFFLOAD_ASYNC=1 SXE_OFFLOAD_ASYNC_WINDOW=0 SXE_OFFLOAD_H2D_KERNEL=1
run async_w2_k0 SXE_OFFLOAD_ASYNC=1 SXE_OFFLOAD_ASYNC_WINDOW=2 SXE_OFFLOAD_H2D_KERNEL=0
run async_w0_k0 SXE_OFFLOAD_ASYNC=1
