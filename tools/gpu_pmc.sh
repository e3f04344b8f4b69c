#!/bin/bash
# rocprofv3 PMC passes (counters only, no traces; each pass within the per-block limits) over the
# hand-written kernels of tools/pmc_kernels.py. Summary: python tools/pmc_summary.py gpurun_out/pmc/*
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
    python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $OUT/$name.log 2>&1
}
run p1 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
 && run p2 FETCH_SIZE GRBM_GUI_ACTIVE \
 && run p3 WRITE_SIZE TCC_HIT_sum
rc=$?
find $OUT -name "*.csv" ! -name "*counter_collection*" -delete
exit $rc
