set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread > gpurun_out/layout_tests.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/layout_bench.json 2> gpurun_out/layout_bench.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/layout_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/layout_prof.log 2>&1
