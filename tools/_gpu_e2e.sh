set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -x -v --timeout 200 --timeout-method thread > gpurun_out/e2e_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_e2e.py 5 8 > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err && \
timeout -k 10 200 python -u tools/bench_components.py 10 heads > gpurun_out/heads_comp.json 2> gpurun_out/heads_comp.err
