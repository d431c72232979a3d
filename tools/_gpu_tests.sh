set -o pipefail
cd $GRAFT_REPO_ROOT
if [ -n "$TESTK" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTK" > gpurun_out/tests.log 2>&1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
fi
