#!/bin/bash
# A/B the training bench under alternative environment settings on one box, interleaved (A B A B ...)
# so clock / thermal drift hits both arms equally.
#   tools/ab_bench.sh OUT_PREFIX ROUNDS "ENV_A" "ENV_B" [bench args...]
# ENV_x: space-separated VAR=VALUE list ("" = defaults). Each run's JSON line goes to OUT_PREFIX.log.
set -o pipefail
out=$1; rounds=$2; ea=$3; eb=$4; shift 4
mkdir -p "$(dirname "$out")"
: > "$out.log"
for i in $(seq 1 "$rounds"); do
  for arm in A B; do
    if [ $arm = A ]; then e=$ea; else e=$eb; fi
    echo "## round $i arm $arm env: $e" >> "$out.log"
    env $e timeout -k 10 300 python bench.py "$@" 2> "$out.$arm.$i.err" | grep '^{' >> "$out.log" || { echo "run failed rc=$?" >> "$out.log"; tail -20 "$out.$arm.$i.err" >> "$out.log"; exit 1; }
  done
done
