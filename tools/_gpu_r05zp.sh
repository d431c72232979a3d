# Round-5 pass on the product tree on the final round-5 tree (library rebuilt after the prefetch A/B revert): whole GPU suite, smoke, default bench
# line, kernel stats of the bench command (live PMC leg off under the tracer), OTF timing
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zp
mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -2 $R/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail $R/smoke.log; exit 3; }
tail -2 $R/smoke.log
timeout -k 10 500 python3 -u bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 4; }
python3 -c "
import json;d=json.loads(open('$R/bench.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])
print('mfma_busy w8', d['roofline_gemm'].get('mfma_busy'), d['roofline_gemm'].get('mfma_counters'))
print('fp32', d['fp32_mode']['value'], d['fp32_mode']['roofline_gemm']['avg_launch_ms'], d['fp32_mode']['roofline_gemm'].get('mfma_busy'), d['fp32_mode']['roofline_lookup']['avg_launch_ms'], d['fp32_mode']['roofline_lookup'].get('traffic_read'))
print('train', d.get('train_step', {}).get('ms_per_step'), d.get('train_step', {}).get('frame_pairs_per_s')); print('highres', d['highres_fs']['otf_ms'], d['highres_fs']['volume_ms']); print('cpu', d['cpu_baseline']['value'])"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --live-pmc off > $R/bench_prof.json 2> $R/bench_prof.err || exit 5
grep -h "corr_lookup\|corr_pyramid\|otf_lookup" $R/prof/*kernel_stats.csv | cut -c1-200
for shape in 2,270,480 8,55,128; do
  OTF_SHAPE=$shape timeout -k 10 180 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/otf_$shape.json 2> $R/otf.err || exit 6
  cat $R/otf_$shape.json
done
find $R -name '*kernel_trace.csv' -size +20M -delete
echo done
