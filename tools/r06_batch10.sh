#!/bin/bash
# Round-6 batch 10: tune the GEMM shapes of the Mixtral-EP step that the packaged TunableOp table lacks
# (expert projections at capacity C, dense projections at 4096 tokens), then A/B the merged table.
set -o pipefail
O=gpurun_out/r06/batch10
mkdir -p $O
cp shuffle_exchange_amd/tuning/tunableop_mi355x.csv $O/packaged.csv
(while sleep 30; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
SXE_GEMM_TUNE_OUT=$O/mixtral_tuned.csv SXE_GEMM_TUNE_MS=150 timeout -k 10 600 python -u bench.py --config mixtral-ep --steps 1 --warmup 1 \
    2>&1 | tee $O/tune_run.log | grep -v "^{" || { tail -30 $O/tune_run.log; exit 1; }
ls -la $O; wc -l $O/mixtral_tuned.csv
for rep in 1 2; do
  for t in packaged tuned; do
    f=$O/packaged.csv; [ $t = tuned ] && f=$O/mixtral_tuned.csv
    SXE_TUNABLEOP_FILE=$f timeout -k 10 300 python bench.py --config mixtral-ep --steps 4 --warmup 2 > $O/ab_${t}_$rep.log 2>&1 \
        || { tail -30 $O/ab_${t}_$rep.log; exit 1; }
    echo "$t rep=$rep $(grep '^{' $O/ab_${t}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
