# flash attention: GPU numerics tests + kernel timings (tools/attn_bench.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_flash_attn_gpu.py tests/test_sparse_attention.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -15 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py 4 > gpurun_out/attn_bench.log 2>&1
rc=$?; cat gpurun_out/attn_bench.log | grep path; exit $rc
