#!/bin/bash
# MX GEMM session: operand-layout probe, kernel tests, bench; then (unless something crashed or
# timed out) the full validation round. Every GPU step has its own time limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
ok_or_fail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/probes/mx_mfma_layout.hip -o /tmp/mx_probe || exit 3
(cd /tmp && cp $GRAFT_REPO_ROOT/tools/probes/mx_layout_check.py . && \
  timeout -k 10 120 python mx_layout_check.py) > gpurun_out/mx_probe.log 2>&1
rc=$?; cat gpurun_out/mx_probe.log; ok_or_fail $rc || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_mx_gemm_gpu.py tests/test_grouped_gemm_q_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mx_tests.log; ok_or_fail $rc || exit $rc
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python tools/mx_gemm_bench.py > gpurun_out/mx_bench.log 2>&1
  rc=$?; cat gpurun_out/mx_bench.log; ok_or_fail $rc || exit $rc
fi
[ "${MX_ONLY:-0}" = "1" ] && exit 0
bash tools/gpu_round.sh
