#!/bin/bash
# Round-6 batch 12: re-tune the headline step's GEMM shapes online with the step's real operands
# (hipBLASLt solutions, 30 ms each) starting from an empty table, then A/B packaged vs re-tuned.
set -o pipefail
O=gpurun_out/r06/batch12
mkdir -p $O
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/packaged.csv
grep '^Validator' $O/packaged.csv > $O/empty.csv
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 SXE_TUNABLEOP_FILE=$O/empty.csv SXE_GEMM_TUNE_OUT=$O/tuned.csv SXE_GEMM_TUNE_MS=30 \
    timeout -k 10 700 python -u bench.py --steps 1 --warmup 1 > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
echo "tuned rows: $(grep -c Gemm $O/tuned.csv)"
for t in packaged retuned packaged retuned; do
  f=$O/packaged.csv; [ $t = retuned ] && f=$O/tuned.csv
  SXE_TUNABLEOP_FILE=$f timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/ab_$t.log 2>&1 \
      || { tail -30 $O/ab_$t.log; exit 1; }
  echo "headline $t $(grep '^{' $O/ab_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
