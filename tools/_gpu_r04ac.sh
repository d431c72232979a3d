# Round-4: FETCH_SIZE / WRITE_SIZE of the chunk-piece RAFT lookup backward at cfg2 b8 (one pass per counter)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ac
mkdir -p $R
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/pmc_$c -o run -- python3 tools/bench_corr_bwd.py 2 bf16 cfg2 > /dev/null 2> $R/pmc_$c.err || { tail -5 $R/pmc_$c.err; exit 2; }
  f=$(find $R/pmc_$c -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_kernel.py $f corr_lookup_backward_kernel
done
