#!/bin/bash
# Round-6 batch 25: tune (hipBLASLt only, 100 ms per solution) the headline GEMM shapes the packaged
# table lacks after the round-6 step changes (new LM-head / QKV layouts), then A/B packaged vs merged.
set -o pipefail
O=gpurun_out/r06/batch25
mkdir -p $O
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/packaged.csv
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 SXE_GEMM_TUNE_OUT=$O/tuned.csv SXE_GEMM_TUNE_MS=100 timeout -k 10 700 \
    python -u bench.py --steps 1 --warmup 1 > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
echo "tuned rows: $(grep -c Gemm $O/tuned.csv)"; grep Gemm $O/tuned.csv | head -20
python tools/merge_tunableop.py $O/tuned.csv > $O/merge.log 2>&1 || { cat $O/merge.log; exit 1; }
cat $O/merge.log
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/merged.csv
diff $O/packaged.csv $O/merged.csv | head -20
for t in packaged merged packaged merged; do
  SXE_TUNABLEOP_FILE=$O/$t.csv timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/ab_$t.log 2>&1 || { tail -30 $O/ab_$t.log; exit 1; }
  echo "headline $t $(grep '^{' $O/ab_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
