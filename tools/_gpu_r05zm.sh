# Round 5: bfloat16 G in the bf16 modes (build writes bf16, GEMMs read it) vs fp32 G (RMD_GRAD_BF16=0);
# parity first, then cfg2 / cfg5 backward timings and kernel stats
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zm
mkdir -p $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_grad_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gb_tests.log 2>&1 || { tail -40 $R/gb_tests.log; exit 2; }
tail -1 $R/gb_tests.log
for rep in 1 2; do
  for gb in 1 0; do
    for cfg in cfg2 cfg5; do
      RMD_GRAD_BF16=$gb timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 bf16 $cfg > $R/cb_bf${gb}_${cfg}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
      python3 -c "import json;d=json.load(open('$R/cb_bf${gb}_${cfg}_$rep.json'));print('corr_bwd bf16G=$gb $cfg $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
cp $R/prof/run_kernel_stats.csv $R/kernel_stats_cfg2_bf16.csv
grep -h "grad_gemm\|grad_build\|pool_targets" $R/prof/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,90), $2}'
find $R -name '*kernel_trace.csv' -delete
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_ctf_l3.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 7; }
tail -1 $R/tests.log
