# Round-4 pass: whole GPU suite, 2-rank gloo rehearsal (live PMC + cpu_baseline at N>1), headline-only
# kernel trace (the 12 lookups + GEMM of bench.py without the extra legs), RAFT volume backward at cfg2
# b8 (kernel trace + FETCH/WRITE passes), cfg5 training-step kernel trace (DAP weight-gradient reduce)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04f
mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -2 $R/tests.log
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --one-device --steps 10 --warmup 3 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --cpu-budget-s 3 > $R/rehearse2.json 2> $R/rehearse2.err || { tail -20 $R/rehearse2.err; exit 3; }
python3 -c "import json;d=json.loads(open('$R/rehearse2.json').read().splitlines()[-1]);print('rehearse2', d['value'],d['n_gpus'],d['roofline']['traffic_source'],d['roofline']['traffic'],d['cpu_baseline']['value'],d['cpu_baseline'].get('note'))"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_head -o run -- python3 bench.py --steps 20 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off > $R/head.json 2> $R/head.err || exit 4
grep -h "corr_lookup\|corr_pyramid\|prep_pair" $R/prof_head/*kernel_stats.csv
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_bwd -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > $R/bwd.json 2> $R/bwd.err || exit 5
cat $R/bwd.json
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/pmc_bwd_$c -o run -- python3 tools/bench_corr_bwd.py 2 bf16 cfg2 > /dev/null 2> $R/pmc_bwd_$c.err || exit 6
done
timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $R/prof_train -o run -- python3 tools/train_probe.py 3 3 > $R/train.log 2>&1 || exit 7
f=$(find $R/prof_train -name '*kernel_trace.csv' | head -1); python3 tools/train_profile_summary.py $f > $R/train_summary.json && head -c 1500 $R/train_summary.json
find $R -name '*kernel_trace.csv' -size +20M -delete
echo done
