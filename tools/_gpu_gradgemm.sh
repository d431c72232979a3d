# grad GEMM (RAFT correlation backward) parity tests + timing + kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-gg}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py -x -q --timeout 200 --timeout-method thread -k "grad or backward" > $O/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 fp32 > $O/${TAG}_bwd.json 2> $O/${TAG}_bwd.err && \
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 tools/bench_corr_bwd.py 5 fp32 > $O/$TAG/prof.log 2>&1
