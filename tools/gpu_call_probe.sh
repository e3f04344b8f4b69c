#!/bin/bash
# MX MFMA layout probe only (one short GPU step).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/probes/mx_mfma_layout.hip -o /tmp/mx_probe || exit 3
cd /tmp && cp $GRAFT_REPO_ROOT/tools/probes/mx_layout_check.py . && \
  timeout -k 10 240 python mx_layout_check.py > $GRAFT_REPO_ROOT/gpurun_out/mx_probe.log 2>&1
rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/mx_probe.log; exit $rc
