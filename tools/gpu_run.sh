#!/bin/bash
# One parameterised GPU-box session (replaces the per-experiment gpu_call_*.sh wrappers).
#
#   gpurun -- bash tools/gpu_run.sh STEP [STEP ...]
#
# STEP is NAME[@VAR=VALUE[@VAR=VALUE...]]: the VAR=VALUE pairs are exported for that step only
# (A/B runs of one step under different SXE_* knobs). Every step runs under its own time limit,
# writes gpurun_out/<NAME>[_<n>].log and the chain stops at the first failure (a crash, abort or
# time-out ends the session: nothing else touches the GPU after it).
#
# NAME                what it runs
#   tests[=f1,f2]     pytest -m gpu over tests/ (or the listed test files)
#   smoke             __graft_entry__.py smoke
#   bench             bench.py ($BENCH_ARGS, default --steps 3 --warmup 1)
#   prof              rocprofv3 --kernel-trace --stats of one bench.py step ($BENCH_ARGS)
#   attn              tools/attn_bench.py ($ATTN_ARGS)
#   attnprof          rocprofv3 kernel stats of tools/attn_bench.py 1
#   pmc_attn          rocprofv3 counter passes over tools/pmc_attn.py
#   pmc               rocprofv3 counter passes over tools/pmc_kernels.py
#   pmcw=SCRIPT       the same kind of counter passes (plus stall counters) over tools/SCRIPT
#   decode            tools/decode_bench.py ($DECODE_ARGS)
#   decodeprof        rocprofv3 kernel trace of eager decode steps
#   paged             tools/paged_attn_bench.py
#   skinny            tools/skinny_bench.py
#   gg                tools/grouped_gemm_bench.py
#   mx                tools/mx_gemm_bench.py ($MX_ARGS)
#   moe               tools/moe_bench.py ($MOE_ARGS)
#   compile           tools/compile_bench.py ($COMPILE_ARGS): DeepCompile compiled vs eager step
#   tune              bounded TunableOp search over the Llama-3-8B GEMM shapes ($TUNE_ARGS)
#   py=SCRIPT         python SCRIPT ($PY_ARGS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PYTHONPATH
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"

pmc_passes() {  # $1 = output dir, $2 = workload script, then "name counters..." passes separated by ';'
  local out=$1 work=$2; shift 2
  mkdir -p "$out"
  local IFS=';'
  for pass in $*; do
    IFS=' ' read -r -a a <<< "$pass"
    timeout -s KILL 120 rocprofv3 --pmc "${a[@]:1}" --output-format csv -d "$out/${a[0]}" -o pmc -- \
      python3 "$work" > "$out/${a[0]}.log" 2>&1 || return $?
  done
  find "$out" -name "*.csv" ! -name "*counter_collection*" -delete
}

run_step() {  # $1 = name, $2 = log file
  local name=$1 log=$2 arg=""
  case "$name" in *=*) arg=${name#*=}; name=${name%%=*} ;; esac
  case "$name" in
    tests)
      local files="tests"; [ -n "$arg" ] && files=$(echo "$arg" | tr ',' ' ')
      timeout -k 10 1100 $PYT $files > "$log" 2>&1 ;;
    smoke) timeout -k 10 300 python __graft_entry__.py smoke > "$log" 2>&1 ;;
    bench) timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > "$log" 2>&1 ;;
    prof)
      local pd=${PROF_DIR:-gpurun_out/prof}
      mkdir -p "$pd"
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$pd" -o bench -- \
        python3 bench.py ${BENCH_ARGS:---steps 1 --warmup 1} > "$log" 2>&1
      local rc=$?; find "$pd" -name "*kernel_trace.csv" -size +50M -delete; return $rc ;;
    attn) timeout -k 10 300 python tools/attn_bench.py ${ATTN_ARGS:-4} > "$log" 2>&1 ;;
    attnprof)
      mkdir -p gpurun_out/attnprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attnprof -o attn -- \
        python3 tools/attn_bench.py ${ATTN_ARGS:-1} > "$log" 2>&1 ;;
    pmc_attn)
      pmc_passes gpurun_out/pmc_attn tools/pmc_attn.py \
        "a1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS;a2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_WAVES;a3 GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT" > "$log" 2>&1 ;;
    pmc)
      pmc_passes gpurun_out/pmc tools/pmc_kernels.py \
        "p1 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES;p2 FETCH_SIZE GRBM_GUI_ACTIVE;p3 WRITE_SIZE TCC_HIT_sum" > "$log" 2>&1 ;;
    pmcw)  # counter passes over an arbitrary workload script: pmcw=tools/pmc_mx.py
      pmc_passes gpurun_out/pmcw tools/$(basename "$arg") \
        "w1 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS;w2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC;w3 FETCH_SIZE GRBM_GUI_ACTIVE;w4 WRITE_SIZE TCC_HIT_sum" > "$log" 2>&1 ;;
    decode) timeout -k 10 700 python tools/decode_bench.py ${DECODE_ARGS:---batches 1,16,64 --modes graphs,graphs+fp8} > "$log" 2>&1 ;;
    decodeprof)
      mkdir -p gpurun_out/decprof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/decprof -o dec -- \
        python3 tools/decode_bench.py --batches ${B:-1} --modes ${MODES:-eager} --steps 16 > "$log" 2>&1
      local rc=$?; find gpurun_out/decprof -name "*kernel_trace.csv" -size +60M -delete; return $rc ;;
    paged) timeout -k 10 300 python tools/paged_attn_bench.py > "$log" 2>&1 ;;
    skinny) timeout -k 10 300 python tools/skinny_bench.py > "$log" 2>&1 ;;
    gg) timeout -k 10 300 python tools/grouped_gemm_bench.py > "$log" 2>&1 ;;
    mx) timeout -k 10 300 python tools/mx_gemm_bench.py ${MX_ARGS} > "$log" 2>&1 ;;
    moe) timeout -k 10 900 python tools/moe_bench.py ${MOE_ARGS} > "$log" 2>&1 ;;
    compile) timeout -k 10 900 python tools/compile_bench.py ${COMPILE_ARGS} > "$log" 2>&1 ;;
    tune) timeout -k 10 ${TUNE_LIMIT:-900} python3 tools/tune_gemms.py gpurun_out/tunableop_llama3_8b.csv ${TUNE_ARGS} \
      > "$log" 2>&1 ;;
    py) timeout -k 10 ${PY_TIMEOUT:-600} python "$arg" ${PY_ARGS} > "$log" 2>&1 ;;
    *) echo "unknown step $name" > "$log"; return 2 ;;
  esac
}

n=0
for spec in "$@"; do
  n=$((n + 1))
  IFS='@' read -r -a parts <<< "$spec"
  name=${parts[0]}
  tag=$(echo "${name%%=*}" | tr -c 'a-zA-Z0-9_\n' '_')
  log=gpurun_out/${tag}_$n.log
  echo "== step $n: $spec -> $log"
  ( for kv in "${parts[@]:1}"; do export "$kv"; done; run_step "$name" "$log" )
  rc=$?
  tail -n ${TAIL:-6} "$log"
  if [ $rc -ne 0 ]; then echo "== step $n failed (exit $rc)"; exit $rc; fi
done
