# Round 5: grad-GEMM register prefetch depth A/B (RMD_GRAD_PF, corr_grad.hip): product (depth 2 on 128-wide
# tiles, 256-wide tiles at depth 1) vs depth 1 everywhere (= previous product) vs 128-wide tiles at depth 1 / 2;
# parity first, then cfg2 / cfg5 bf16 backward timings
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zo
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_grad_build.py tests/test_gpu_corr.py tests/test_gpu_ctf_l3.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for rep in 1 2; do
  for v in product pf1 pf2tn128 pf1tn128; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    for cfg in cfg2 cfg5; do
      RMD_LIBRARY=$L timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 bf16 $cfg > $R/cb_${v}_${cfg}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
      python3 -c "import json;d=json.load(open('$R/cb_${v}_${cfg}_$rep.json'));print('corr_bwd $v $cfg $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg5 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
cp $R/prof/run_kernel_stats.csv $R/kernel_stats_cfg5_bf16.csv
grep -h "grad_gemm\|grad_build" $R/prof/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,90), $2}'
find $R -name '*kernel_trace.csv' -delete
echo done
