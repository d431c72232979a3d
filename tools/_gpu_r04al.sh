# Round-4: OTF operand segments through LDS (product) vs per-lane strided reads (segold): OTF GPU tests,
# bitwise comparison of cfg2 outputs / gradients, kernel stats of the 4K leg per build
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04al
mkdir -p $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_otf.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for p in bf16 fp32; do
  timeout -k 10 120 python3 tools/otf_bwd_dump.py $R/new_$p.npz $p && RMD_LIBRARY=$PWD/tools/_ab/librmd_segold.so timeout -k 10 120 python3 tools/otf_bwd_dump.py $R/old_$p.npz $p || exit 3
  python3 -c "
import numpy as np; a=np.load('$R/new_$p.npz'); b=np.load('$R/old_$p.npz')
print('$p bitwise equal:', all(np.array_equal(a[k], b[k]) for k in ('g1','g2')))"
done
for v in product segold; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/p_$v -o run -- python3 tools/bench_otf.py --reps 3 --cfg2-off > $R/b_$v.json 2> $R/b_$v.err || { tail $R/b_$v.err; exit 4; }
  python3 - $R/p_$v/run_kernel_stats.csv $v $R/b_$v.json <<'PY'
import csv, json, sys
k = {r["Name"][28:60]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e3, 1)) for r in csv.DictReader(open(sys.argv[1])) if "segments" in r["Name"] or "otf_lookup" in r["Name"]}
print(sys.argv[2], json.load(open(sys.argv[3]))["highres_4k"]["otf_ms"], k)
PY
done
rm -f $R/*.npz; find $R -name '*kernel_trace.csv' -delete
