#!/bin/bash
# Round-6 measurement batch 6: decode KV-split floor (SXE_PA_MIN_KEYS) x merge placement (fused into the
# o_proj prologue vs a merge launch) at batch 1 / 8 / 32, ctx 1024 and 4096; MX auto tile on small M.
set -o pipefail
O=gpurun_out/r06/batch6
mkdir -p $O
dec() {  # name, ctx, env...
  local name=$1 ctx=$2; shift 2
  env "$@" timeout -k 10 300 python tools/decode_bench.py --batches 1,8,32 --ctx $ctx --modes graphs > $O/decode_$name.log 2>&1 \
      || { echo "decode $name failed"; tail -30 $O/decode_$name.log; exit 1; }
  echo "decode $name"; grep '^{' $O/decode_$name.log
}
timeout -k 10 300 python -u -m pytest tests/test_mx_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/mx_tests.log 2>&1 || { tail -30 $O/mx_tests.log; exit 1; }
tail -1 $O/mx_tests.log
timeout -k 10 240 python tools/mx_gemm_bench.py --quick --shapes "512,4096,4096;512,14336,4096;128,14336,4096;256,4096,4096;1024,4096,4096;512,6144,4096;1024,6144,4096;2048,6144,4096" > $O/mx_auto.log 2>&1 || { tail -20 $O/mx_auto.log; exit 1; }
grep "M=" $O/mx_auto.log | sed 's/| FPx.*//'
dec fused_k64 1024 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=64 && \
dec fused_k128 1024 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=128 && \
dec fused_k256 1024 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=256 && \
dec sep_k64 1024 SXE_DECODE_FUSE_ATTN=0 SXE_PA_MIN_KEYS=64 && \
dec sep_k128 1024 SXE_DECODE_FUSE_ATTN=0 SXE_PA_MIN_KEYS=128 && \
dec sep_k256 1024 SXE_DECODE_FUSE_ATTN=0 SXE_PA_MIN_KEYS=256 && \
dec fused_k64_c4k 4096 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=64 && \
dec fused_k128_c4k 4096 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=128 && \
dec fused_k256_c4k 4096 SXE_DECODE_FUSE_ATTN=1 SXE_PA_MIN_KEYS=256 && \
dec sep_k128_c4k 4096 SXE_DECODE_FUSE_ATTN=0 SXE_PA_MIN_KEYS=128
