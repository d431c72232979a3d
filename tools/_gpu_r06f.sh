# Round 6: default bench line twice (timed legs before the profiling children)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06f
mkdir -p $R
for i in 1 2; do
timeout -k 10 600 python3 -u bench.py > $R/bench_$i.json 2> $R/bench_$i.err || { tail -20 $R/bench_$i.err; exit 4; }
python3 -c "
import json;d=json.loads(open('$R/bench_$i.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'], 'busy', d['roofline_gemm'].get('mfma_busy'))
f=d['fp32_mode']; print('fp32', f['value'], f['ms_per_step'], f['roofline_gemm']['avg_launch_ms'], f['roofline_gemm'].get('mfma_busy'), f['roofline_gemm'].get('mfma_counters',{}).get('clock_ghz'), f['roofline_lookup']['avg_launch_ms'])"
done
echo done
