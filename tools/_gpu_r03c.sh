# OTF occupancy/shape A/B + GPU tests of every path whose launcher was cleaned (DICL, DAP, warp, OTF, corr)
set -o pipefail
R=gpurun_out/r03c
mkdir -p $R
run() { RMD_LIBRARY=$1 timeout -k 10 300 python3 -u tools/otf_time.py 10 >> $R/otf_ab.jsonl 2>> $R/err.log; }
rm -f $R/otf_ab.jsonl
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 3
for v in b1o2 b1o4 b2o2; do run $PWD/tools/_bin/librmd_otf_$v.so || exit 4; done
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 5
cat $R/otf_ab.jsonl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 6; }
tail -2 $R/tests.log
