# Round-4 first pass: store-pattern microbenchmarks (lookup output, GEMM level 0 incl. 2x8 chunks), lookup
# ablations (stores / loads dropped), kernel trace of the 12 headline lookups, OTF GPU tests (deterministic
# backward) and OTF timing
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04b
mkdir -p $R
timeout -k 10 60 tools/_ab/lookup_store_bench > $R/lookup_store_bench.jsonl 2>&1 || exit 2
timeout -k 10 60 tools/_ab/store_pattern_bench > $R/store_pattern_bench.jsonl 2>&1 || exit 3
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/lookup_time.py 20 bf16 >> $R/lookup_ab.jsonl 2>> $R/err.log; }
run $P || exit 4
for v in abl1 abl2 abl3; do run $PWD/tools/_ab/librmd_$v.so || exit 5; done
run $P || exit 6
cat $R/lookup_store_bench.jsonl $R/store_pattern_bench.jsonl $R/lookup_ab.jsonl
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/lookup_time.py 20 bf16 > $R/prof.log 2>&1 || exit 7
find $R/prof -name '*kernel_stats.csv' -exec grep -h corr_lookup {} \;
timeout -k 10 400 python -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/otf_tests.log 2>&1 || { tail -30 $R/otf_tests.log; exit 8; }
tail -2 $R/otf_tests.log
