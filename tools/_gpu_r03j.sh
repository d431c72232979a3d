# x3 (fp32-mode) GEMM A/B: product vs stores dropped (abl1), epilogue only (abl2), L2-hot B (bhot, bhot+abl1)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r03j
mkdir -p $R
rm -f $R/x3_ab.jsonl
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/x3_time.py ${REPS:-20} ${PREC:-fp32} >> $R/x3_ab.jsonl 2>> $R/err.log; }
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
B=$PWD/tools/_bin
run $P || exit 3
for v in $VARIANTS; do run $B/librmd_$v.so || exit 4; done
run $P || exit 5
cat $R/x3_ab.jsonl
