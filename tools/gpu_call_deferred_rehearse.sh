cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_deferred_comm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/deferred_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/deferred_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=" " bash tools/rehearse_configs.sh
