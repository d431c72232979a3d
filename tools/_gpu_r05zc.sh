# Round 5: G build v3 (LDS slot tile) parity + diagnostics, then grad-GEMM split cap A/B (1 / 2 / 4 vs 8)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zc
mkdir -p $R
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_grad_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gb_tests.log 2>&1 || { tail -30 $R/gb_tests.log; exit 2; }
tail -2 $R/gb_tests.log
bash tools/_gpu_r05za.sh r05zc/za || exit 3
for rep in 1 2; do
  for v in product ggs1 ggs2 ggs4; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 bf16 cfg2 > $R/cb_${v}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
    python3 -c "import json;d=json.load(open('$R/cb_${v}_$rep.json'));print('corr_bwd $v bf16 $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
  done
done
for v in ggs1 ggs2; do
  RMD_LIBRARY=$PWD/tools/_ab/librmd_$v.so timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$v -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
  grep -h "grad_gemm\|grad_build" $R/prof_$v/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,70), $2}'
done
find $R -name '*kernel_trace.csv' -delete
