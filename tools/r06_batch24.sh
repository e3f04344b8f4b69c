#!/bin/bash
# Round-6 batch 24 (final tree): smoke + whole GPU suite, then the headline bench as the driver runs it.
set -o pipefail
bash tools/r06_suite.sh || exit 1
O=gpurun_out/r06/batch24
mkdir -p $O
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/headline_20steps.log 2>&1 || { tail -30 $O/headline_20steps.log; exit 1; }
grep '^{' $O/headline_20steps.log | cut -c1-300
