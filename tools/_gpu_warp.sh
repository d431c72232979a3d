set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_warp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/warp_tests.log 2>&1
