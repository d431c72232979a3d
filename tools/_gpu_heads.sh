set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_heads.py -x -v --timeout 120 --timeout-method thread > gpurun_out/heads_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_components.py 20 heads > gpurun_out/heads_comp.json 2> gpurun_out/heads_comp.err && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/all_tests.log 2>&1
