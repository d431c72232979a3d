# Round-4 lookup A/B, same box, events per launch + output checksum (bitwise-equal outputs expected):
# base (round-3 source), wm (word-mask padding, the current source), h64 (+ b64 half-row loads),
# xst (+ LDS-transposed 16-B stores), xsth64 (both); kernel trace of h64 and xsth64
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04d
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
B=$PWD/tools/_ab
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/lookup_time.py 30 bf16 >> $R/lookup_ab.jsonl 2>> $R/err.log; }
run $B/librmd_base.so || exit 3
run $P || exit 4
for v in h64 xst xsth64; do run $B/librmd_$v.so || exit 5; done
run $B/librmd_base.so || exit 6
for v in xsth64 h64; do run $B/librmd_$v.so || exit 7; done
run $P || exit 8
cat $R/lookup_ab.jsonl
for v in base h64 xsth64; do
RMD_LIBRARY=$B/librmd_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$v -o run -- python3 tools/lookup_time.py 20 bf16 > $R/prof_$v.log 2>&1 || exit 9
echo "== $v"; find $R/prof_$v -name '*kernel_stats.csv' -exec grep -h corr_lookup {} \;
done
