# Round-4: kernel stats of the 4K on-the-fly inference leg (bench_otf highres part only)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ak
mkdir -p $R
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_otf.py --reps 3 --cfg2-off > $R/b.json 2> $R/b.err || { tail $R/b.err; exit 2; }
python3 - $R/prof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 2))
PY
find $R -name '*kernel_trace.csv' -delete
