# rocprofv3 kernel trace of Llama-3-8B decode (batch 1, eager engine steps -> per-kernel durations)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/decprof && export PYTHONPATH=$PWD
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/decprof -o dec -- \
  python3 tools/decode_bench.py --batches ${B:-1} --modes ${MODES:-eager} --steps 16 > gpurun_out/decprof/run.log 2>&1
rc=$?; tail -2 gpurun_out/decprof/run.log; find gpurun_out/decprof -name "*kernel_trace.csv" -size +60M -delete; exit $rc
