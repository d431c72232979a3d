# Round-4 lookup bound: output-store pattern microbenchmark, then the product lookup vs stores-dropped /
# loads-dropped / both builds (same instruction stream, kOOB offsets), events per launch, and a kernel
# trace of the product's 12 headline lookups alone
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04a
mkdir -p $R
timeout -k 10 60 tools/_ab/lookup_store_bench > $R/store_bench.jsonl 2>&1 || exit 2
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/lookup_time.py 20 bf16 >> $R/lookup_ab.jsonl 2>> $R/err.log; }
run $P || exit 3
for v in abl1 abl2 abl3; do run $PWD/tools/_ab/librmd_$v.so || exit 4; done
run $P || exit 5
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/lookup_time.py 20 bf16 > $R/prof.log 2>&1 || exit 6
cat $R/store_bench.jsonl $R/lookup_ab.jsonl
find $R/prof -name '*kernel_stats.csv' -exec grep -h corr_lookup {} \;
