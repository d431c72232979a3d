# Round-4: RAFT backward GEMMs, interleaved chunk schedule (ggilv) vs product: grad tests, kernel stats of
# tools/bench_corr_bwd.py at cfg2 b8 per build
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ad
mkdir -p $R
RMD_LIBRARY=$PWD/tools/_ab/librmd_ggilv.so timeout -k 10 400 python -u -m pytest tests/test_gpu_corr.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for v in product ggilv product ggilv; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  rm -rf $R/p_$v
  RMD_LIBRARY=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/p_$v -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > $R/b_$v.json 2> $R/b_$v.err || { tail $R/b_$v.err; exit 3; }
  python3 - $R/p_$v/run_kernel_stats.csv $v $R/b_$v.json <<'PY'
import csv, json, sys
k = {r["Name"][:48]: round(float(r["AverageNs"]) / 1e3, 1) for r in csv.DictReader(open(sys.argv[1])) if "grad_gemm" in r["Name"]}
print(sys.argv[2], json.load(open(sys.argv[3]))["backward_ms"], k)
PY
done
find $R -name '*kernel_trace.csv' -delete
