#!/bin/bash
# Round-6 measurement batch 4: (a) llama70b-infinity synchronous vs asynchronous host tier with the
# piecewise grad D2H; (b) batch-1 decode: o_proj-fused split merge vs separate merge, KV split targets.
set -o pipefail
O=gpurun_out/r06/batch4
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" SXE_OFFLOAD_TRACE=1 timeout -k 10 400 python bench.py --config llama70b-infinity --steps 4 --warmup 2 \
      > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'])"
}
dec() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/decode_bench.py --batches 1,8 --modes graphs > $O/decode_$name.log 2>&1 \
      || { echo "decode $name failed"; tail -30 $O/decode_$name.log; exit 1; }
  echo "decode $name"; tail -4 $O/decode_$name.log
}
run sync SXE_OFFLOAD_ASYNC=0 && \
run async_w0_k0 SXE_OFFLOAD_ASYNC=1 && \
run async_w2_k1 SXE_OFFLOAD_ASYNC=1 SXE_OFFLOAD_ASYNC_WINDOW=2 SXE_OFFLOAD_H2D_KERNEL=1 && \
dec fused SXE_DECODE_FUSE_ATTN=1 && \
dec separate_mergelaunch SXE_DECODE_FUSE_ATTN=0 SXE_PA_LAST_MERGE=0 && \
dec separate_lastmerge SXE_DECODE_FUSE_ATTN=0 SXE_PA_LAST_MERGE=1 && \
dec lastmerge_t256 SXE_DECODE_FUSE_ATTN=0 SXE_PA_LAST_MERGE=1 SXE_PA_TARGET_WGS=256 && \
dec lastmerge_k128 SXE_DECODE_FUSE_ATTN=0 SXE_PA_LAST_MERGE=1 SXE_PA_MIN_KEYS=128 && \
dec fused_k128 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=128
