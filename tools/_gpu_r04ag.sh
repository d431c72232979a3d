# Round-4 final tree: 2-rank gloo rehearsal on one GPU (live PMC + cpu_baseline at N = 2) and the
# headline-only kernel trace (bench.py with the extra legs off) for the lookup / GEMM launch averages
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ag
mkdir -p $R
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --one-device --steps 10 --warmup 3 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --cpu-budget-s 3 > $R/rehearse2.json 2> $R/rehearse2.err || { tail -20 $R/rehearse2.err; exit 3; }
python3 -c "import json;d=json.loads(open('$R/rehearse2.json').read().splitlines()[-1]);print('rehearse2', d['value'],d['n_gpus'],d['roofline']['traffic_source'][:60],d['roofline']['traffic'],d['cpu_baseline']['value'],d['cpu_baseline'].get('note'))"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_head -o run -- python3 bench.py --steps 20 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off > $R/head.json 2> $R/head.err || exit 4
python3 -c "import json;d=json.loads(open('$R/head.json').read().splitlines()[-1]);print('head', d['value'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])"
grep -h "corr_lookup\|corr_pyramid\|prep_pair" $R/prof_head/*kernel_stats.csv | cut -c1-160
find $R -name '*kernel_trace.csv' -delete
