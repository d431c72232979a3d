# Round-4: RAFT lookup backward, whole-chunk vector RMW (product) vs one float per target (vec0): GPU corr
# tests, then kernel stats of tools/bench_corr_bwd.py at cfg2 b8 per build
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04aa
mkdir -p $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for v in product vec0 product vec0; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  rm -rf $R/p_$v
  RMD_LIBRARY=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/p_$v -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > $R/b_$v.json 2> $R/b_$v.err || { tail $R/b_$v.err; exit 3; }
  echo "$v $(cat $R/b_$v.json | head -c 300)"
  grep -h "corr_lookup_backward" $R/p_$v/*kernel_stats.csv | cut -d, -f1-5
done
find $R -name '*kernel_trace.csv' -delete
