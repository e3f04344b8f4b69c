#!/bin/bash
# Round-6 batch 11: tune (hipBLASLt solutions only, 30 ms per solution) the GEMM shapes the packaged
# TunableOp table lacks for one config (one step), merge them into the table, A/B original vs merged.
#   tools/r06_batch11.sh CONFIG
set -o pipefail
cfg=$1
O=gpurun_out/r06/batch11_$cfg
mkdir -p $O
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/packaged.csv
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 SXE_GEMM_TUNE_OUT=$O/tuned.csv SXE_GEMM_TUNE_MS=30 timeout -k 10 700 \
    python -u bench.py --config $cfg --steps 1 --warmup 1 > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
echo "$cfg tuned rows: $(grep -c Gemm $O/tuned.csv)"
python tools/merge_tunableop.py $O/tuned.csv
for t in packaged merged packaged merged; do
  if [ $t = packaged ]; then export SXE_TUNABLEOP_FILE=$O/packaged.csv; else unset SXE_TUNABLEOP_FILE; fi
  timeout -k 10 400 python bench.py --config $cfg --steps 4 --warmup 2 > $O/ab_$t.log 2>&1 \
      || { tail -30 $O/ab_$t.log; exit 1; }
  echo "$cfg $t $(grep '^{' $O/ab_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
