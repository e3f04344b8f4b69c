#!/bin/bash
# rocprofv3 PMC passes over the flash-attention kernels only (tools/pmc_attn.py), counters only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_attn
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
    python3 $GRAFT_REPO_ROOT/tools/pmc_attn.py > $OUT/$name.log 2>&1
}
run a1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
 && run a2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_WAVES \
 && run a3 GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT
rc=$?
find $OUT -name "*.csv" ! -name "*counter_collection*" -delete
exit $rc
