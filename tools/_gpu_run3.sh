set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1s2_tests3.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/r1s2_bench3.json 2> gpurun_out/r1s2_bench3.err
