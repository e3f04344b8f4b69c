# paged attention: GPU numerics tests + kernel timings + decode bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_paged_attention_gpu.py tests/test_decode_graphs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/paged_tests.log 2>&1
rc=$?; tail -15 gpurun_out/paged_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/paged_attn_bench.py > gpurun_out/paged_attn_bench.log 2>&1
rc=$?; grep '"B"' gpurun_out/paged_attn_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/decode_bench.py ${DECODE_ARGS} > gpurun_out/decode_bench.log 2>&1
rc=$?; tail -4 gpurun_out/decode_bench.log; exit $rc
