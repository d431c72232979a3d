# Round 6 full pass on the current tree: whole GPU suite, smoke, default bench line (live PMC legs on),
# kernel stats of the bench command (live PMC off under the tracer)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06e}
mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -2 $R/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail $R/smoke.log; exit 3; }
tail -3 $R/smoke.log
timeout -k 10 600 python3 -u bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 4; }
python3 -c "
import json;d=json.loads(open('$R/bench.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])
print('mfma_busy w8', d['roofline_gemm'].get('mfma_busy'))
f=d['fp32_mode']; print('fp32', f['value'], f['ms_per_step'], f['roofline_gemm']['avg_launch_ms'], f['roofline_gemm'].get('mfma_busy'), f['roofline_gemm'].get('mfma_counters',{}).get('clock_ghz'), f['roofline_lookup']['avg_launch_ms'])
print('train', d.get('train_step', {}).get('ms_per_step')); print('highres', d['highres_fs'].get('otf_ms'), d['highres_fs'].get('volume_ms')); print('cpu', d['cpu_baseline']['value'])"
timeout -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --live-pmc off > $R/bench_prof.json 2> $R/bench_prof.err || exit 5
python3 -c "
import csv,glob
f=glob.glob('$R/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if any(k in n for k in ('corr_lookup_kernel','corr_pyramid','prep_')): print(n[:90], r['Calls'], r['AverageNs'])"
find $R -name '*kernel_trace.csv' -size +20M -delete
echo done
