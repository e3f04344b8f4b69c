#!/bin/bash
# Round-6 batch 3: MX GEMM tile sweep on the shapes where W8A8 lost to bf16 (QKV 2048x6144, small M)
set -o pipefail
O=gpurun_out/r06/mx
mkdir -p $O
for t in 0 1 2 5 7; do
  SXE_MX_TILE=$t timeout -k 10 240 python tools/mx_gemm_bench.py --quick --shapes "2048,6144,4096;512,4096,4096;2048,4096,4096;4096,6144,4096;512,14336,4096" > $O/tile_$t.log 2>&1 || { tail -20 $O/tile_$t.log; exit 1; }
done
timeout -k 10 300 python tools/mx_gemm_bench.py > $O/full_default.log 2>&1
