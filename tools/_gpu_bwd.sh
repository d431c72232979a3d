# RAFT correlation backward: parity tests, then forward/backward timing + kernel stats at cfg5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-bwd}
R=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_corr.py tests/test_gpu_ctf_l3.py tests/test_gpu_e2e.py} > $R/tests.log 2>&1 || exit 3
timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 20 fp32 > $R/corr_bwd_fp32.json 2> $R/corr_bwd.err || exit 4
timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 20 bf16 > $R/corr_bwd_bf16.json 2>> $R/corr_bwd.err || exit 5
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_bwd -o run -- python3 tools/bench_corr_bwd.py 5 fp32 > $R/prof_bwd.log 2>&1 || exit 6
find $R -name "*kernel_trace.csv" -delete
echo done
