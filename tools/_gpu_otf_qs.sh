# OTF lookup query-block shape A/B: product (bf16 16x4, x3 16x2) vs variants, one box
set -o pipefail
R=gpurun_out/otf_qs
mkdir -p $R
run() { RMD_LIBRARY=$1 timeout -k 10 300 python3 -u tools/otf_time.py 10 >> $R/ab.jsonl 2>> $R/err.log; }
rm -f $R/ab.jsonl
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 3
run $PWD/tools/_bin/librmd_otf_b1o2.so || exit 4
run $PWD/tools/_bin/librmd_otf_b1o4.so || exit 5
run $PWD/tools/_bin/librmd_otf_b2o2.so || exit 8
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 6
cat $R/ab.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 7; }
tail -2 $R/tests.log
