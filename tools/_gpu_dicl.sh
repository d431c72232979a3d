set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dicl.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dicl_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_components.py 10 > gpurun_out/comp_all.json 2> gpurun_out/comp_all.err
