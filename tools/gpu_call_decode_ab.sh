cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/decode_bench.py --batches 1,16 --modes graphs,graphs+fp8 > gpurun_out/ab_on.log 2>&1 && \
SXE_DECODE_FUSE_ATTN=0 timeout -k 10 300 python -u tools/decode_bench.py --batches 1,16 --modes graphs,graphs+fp8 > gpurun_out/ab_off.log 2>&1 && \
timeout -k 10 300 python -u tools/decode_bench.py --batches 1,16 --modes graphs,graphs+fp8 > gpurun_out/ab_on2.log 2>&1
rc=$?; for f in ab_on ab_off ab_on2; do echo "== $f"; grep mode gpurun_out/$f.log; done; exit $rc
