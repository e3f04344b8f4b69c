#!/bin/bash
# Round-6 late GPU suite: smoke(), then the whole `pytest -m gpu` suite.
set -o pipefail
O=gpurun_out/r06/suite
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 \
    || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
