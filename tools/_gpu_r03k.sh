# OTF patch-buffer lookup: GPU OTF tests on the product build, then block-shape A/B vs the band kernel
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r03k
mkdir -p $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -2 $R/tests.log
rm -f $R/otf_ab.jsonl
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/otf_time.py 10 $PRECS >> $R/otf_ab.jsonl 2>> $R/err.log; }
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
B=$PWD/tools/_bin
run $P || exit 3
for v in $VARIANTS; do run $B/librmd_$v.so || exit 4; done
run $P || exit 5
cat $R/otf_ab.jsonl
