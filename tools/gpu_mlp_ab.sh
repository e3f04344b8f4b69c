set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof2
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_mlp_tn.py tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_mlp.log 2>&1 \
 && timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_mlp.log 2>&1 \
 && SXE_MLP_TN=0 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_nomlp.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o bench -- \
      python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench2.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_mlp.log; tail -1 gpurun_out/bench_mlp.log; tail -1 gpurun_out/bench_nomlp.log
exit $rc
