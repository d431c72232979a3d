# OTF lookup query-block shape A/B (32x1 product vs 16x2) + OTF GPU tests on the product library
set -o pipefail
R=gpurun_out/otf_qrow
mkdir -p $R
timeout -k 10 300 python3 -u tools/otf_time.py 10 > $R/p1.json 2> $R/err.log || { tail $R/err.log; exit 3; }
RMD_LIBRARY=$PWD/tools/_bin/librmd_otf16x2.so timeout -k 10 300 python3 -u tools/otf_time.py 10 > $R/v16x2.json 2>> $R/err.log || exit 4
timeout -k 10 300 python3 -u tools/otf_time.py 10 > $R/p2.json 2>> $R/err.log || exit 5
cat $R/p1.json $R/v16x2.json $R/p2.json
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 6; }
tail -2 $R/tests.log
