# Round 6: the balanced-schedule whole-pyramid test and the S24 / cfg2 corr tests
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06i
mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_corr.py -m gpu -x -v -k "x3_balanced or s24 or cfg2 or cfg1" --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
grep -E "PASS|FAIL|passed|failed" $R/tests.log | tail -25
