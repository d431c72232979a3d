# Round-4: OTF backward kernel with its fp64 dP atomic adds skipped (bwdabl, wrong results) vs product,
# kernel stats of the cfg2 training leg
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04an
mkdir -p $R
for v in product bwdabl; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/p_$v -o run -- python3 tools/bench_otf.py --reps 3 --skip-4k > $R/b_$v.json 2> $R/b_$v.err || { tail $R/b_$v.err; exit 4; }
  python3 - $R/p_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
k = {r["Name"][39:68]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e6, 3)) for r in csv.DictReader(open(sys.argv[1])) if "otf_backward" in r["Name"]}
print(sys.argv[2], k)
PY
done
find $R -name '*kernel_trace.csv' -delete
