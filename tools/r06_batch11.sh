#!/bin/bash
# Round-6 batch 11: tune the GEMM shapes the packaged TunableOp table lacks for the SP-32k and the
# 70B-Infinity configs (one step each), merge them into the table, A/B original vs merged.
set -o pipefail
O=gpurun_out/r06/batch11
mkdir -p $O
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/packaged.csv
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for cfg in llama8b-sp32k llama70b-infinity; do
  SXE_GEMM_TUNE_OUT=$O/${cfg}_tuned.csv SXE_GEMM_TUNE_MS=150 timeout -k 10 600 python -u bench.py --config $cfg --steps 1 --warmup 1 \
      > $O/tune_$cfg.log 2>&1 || { tail -30 $O/tune_$cfg.log; exit 1; }
  echo "$cfg tuned rows: $(grep -c Gemm $O/${cfg}_tuned.csv)"
  python tools/merge_tunableop.py $O/${cfg}_tuned.csv
done
for cfg in llama8b-sp32k llama70b-infinity; do
  for t in packaged merged; do
    if [ $t = packaged ]; then export SXE_TUNABLEOP_FILE=$O/packaged.csv; else unset SXE_TUNABLEOP_FILE; fi
    timeout -k 10 400 python bench.py --config $cfg --steps 4 --warmup 2 > $O/ab_${cfg}_$t.log 2>&1 \
        || { tail -30 $O/ab_${cfg}_$t.log; exit 1; }
    echo "$cfg $t $(grep '^{' $O/ab_${cfg}_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
unset SXE_TUNABLEOP_FILE
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/merged.csv
