#!/bin/bash
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/gemm_step_table.py > $O/gemm_step_table.md 2> $O/gemm_step_table.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/decode_prof -o run -- python tools/decode_bench.py --batches 1 --modes graphs --steps 64 > $O/decode_prof.log 2>&1 || exit 1
