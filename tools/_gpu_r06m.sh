# Round 6 final pass: whole GPU suite, smoke, default bench line, rocprofv3 kernel stats of the default
# bench command and of the headline-only command (whose lookup / GEMM averages are the events' kernels),
# x3 SQ counters (MFMA busy, clock) of the product
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06m}
mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -2 $R/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail $R/smoke.log; exit 3; }
tail -3 $R/smoke.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 4; }
python3 -c "
import json;d=json.loads(open('$R/bench.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'], 'busy', d['roofline_gemm'].get('mfma_busy'))
f=d['fp32_mode']; print('fp32', f['value'], f['ms_per_step'], f['roofline_gemm']['avg_launch_ms'], f['roofline_gemm']['mfma_frac'], f['roofline_gemm'].get('mfma_busy'), f['roofline_gemm'].get('mfma_counters',{}).get('clock_ghz'), f['roofline_lookup']['avg_launch_ms'])
print('train', d.get('train_step', {}).get('ms_per_step'), 'hybrid', d.get('hybrid_inference',{}).get('frame_pairs_per_s'), 'dicl', d.get('dicl_matching',{}).get('frame_pairs_per_s'), 'model', d.get('model_level',{}).get('frame_pairs_per_s')); print('highres', d['highres_fs'].get('otf_ms'), d['highres_fs'].get('volume_ms')); print('cpu', d['cpu_baseline']['value'])"
timeout -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --live-pmc off --steps 20 --warmup 5 > $R/bench_prof.json 2> $R/bench_prof.err || exit 5
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_hl -o run -- python3 bench.py $HL --steps 20 --warmup 5 > $R/bench_hl.json 2> $R/bench_hl.err || exit 6
for d in prof prof_hl; do
python3 -c "
import csv,glob
f=glob.glob('$R/$d/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if any(k in n for k in ('corr_lookup_kernel','corr_pyramid','prep_')): print('$d', n[:80], r['Calls'], r['AverageNs'])"
done
python3 -c "
import json;d=json.loads(open('$R/bench_hl.json').read().splitlines()[-1])
print('hl events', d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'], d['fp32_mode']['roofline_gemm']['avg_launch_ms'], d['fp32_mode']['roofline_lookup']['avg_launch_ms'])"
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for pass in A B; do
  eval C=\$SQ$pass
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/p_x3_$pass -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_x3_$pass.err || { tail -5 $R/p_x3_$pass.err; exit 7; }
  python3 tools/pmc_clock.py $R/p_x3_$pass corr_pyramid_x3 x3_product_$pass | tee -a $R/summary.jsonl
done
find $R -name '*kernel_trace.csv' -size +20M -delete
echo done
