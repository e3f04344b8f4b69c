#!/bin/bash
# Round-6 final evidence: smoke(), then every BASELINE config at N=1 back to back on one box.
set -o pipefail
O=gpurun_out/r06/final
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" \
    > $O/wgrad_tests.log 2>&1 || { tail -30 $O/wgrad_tests.log; exit 1; }
tail -1 $O/wgrad_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
echo "smoke ok"
for cfg in llama8b-z3 mixtral-ep llama8b-sp32k llama70b-infinity; do
  timeout -k 10 500 python bench.py --config $cfg --steps 6 --warmup 2 > $O/$cfg.log 2>&1 || { tail -30 $O/$cfg.log; exit 1; }
  echo "$cfg $(grep '^{' $O/$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", d.get("tflops_per_gpu"), "TF", d.get("peak_mem_gb"), "GB")')"
done
