# Round-4 mid-round pass: smoke, default bench line (all legs), OTF timing, OTF backward timing
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04r
mkdir -p $R
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail $R/smoke.log; exit 2; }
tail -2 $R/smoke.log
timeout -k 10 500 python3 -u bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 3; }
python3 -c "
import json;d=json.loads(open('$R/bench.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'], d['roofline_gemm']['mfma_frac'])
print('fp32', d['fp32_mode']['value'], d['fp32_mode']['roofline_gemm']['avg_launch_ms'])
for k in ('model_level','dicl_matching','hybrid_inference','train_step'): print(k, {kk: d[k].get(kk) for kk in ('frame_pairs_per_s','ms_per_step','ms_per_batch','error')})
print('highres', d['highres_fs']); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 150 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/otf_time.json 2> $R/otf_time.err || exit 4
cat $R/otf_time.json
