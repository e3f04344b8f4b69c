#!/bin/bash
# Round-6 measurement batch 5: MX GEMM small-problem tiles (64x128 / 64x64) against the 128x128 tile
# on shapes whose 128x128 grid leaves CUs idle; the tile-variant numerics tests first.
set -o pipefail
O=gpurun_out/r06/mx_small
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mx_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SH="512,4096,4096;512,14336,4096;128,14336,4096;256,4096,4096;1024,4096,4096;512,6144,4096;1024,6144,4096;2048,6144,4096"
for t in 1 9 10 7; do
  SXE_MX_TILE=$t timeout -k 10 240 python tools/mx_gemm_bench.py --quick --shapes "$SH" > $O/tile_$t.log 2>&1 \
      || { tail -20 $O/tile_$t.log; exit 1; }
done
grep -h "SXE_MX_TILE\|M=" $O/tile_*.log | sed 's/| FPx.*//'
dec() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/decode_bench.py --batches 1 --modes graphs > $O/decode_$name.log 2>&1 \
      || { echo "decode $name failed"; tail -30 $O/decode_$name.log; exit 1; }
  echo "decode $name $(grep '^{' $O/decode_$name.log | tail -1)"
}
