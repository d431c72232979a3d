# Round 5: G build with lookup groups (BG = 4 product vs 1 / 2) and the grad-GEMM split rule with
# workspace cost (product) vs the round-4 rule (ggold); parity first
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zd
mkdir -p $R
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_grad_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gb_tests.log 2>&1 || { tail -30 $R/gb_tests.log; exit 2; }
tail -1 $R/gb_tests.log
for v in product bg1 bg2; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/bench_grad_build.py 20 > $R/gb_$v.jsonl 2> $R/gb.err || { tail -5 $R/gb.err; exit 3; }
  echo "== $v"; cat $R/gb_$v.jsonl
done
for rep in 1 2; do
  for v in product ggold; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    for cfg in cfg2 cfg5; do
      for p in bf16 fp32; do
        RMD_LIBRARY=$L timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 $p $cfg > $R/cb_${v}_${cfg}_${p}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
        python3 -c "import json;d=json.load(open('$R/cb_${v}_${cfg}_${p}_$rep.json'));print('corr_bwd $v $cfg $p $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
      done
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
grep -h "grad_gemm\|grad_build\|pool_targets" $R/prof/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,70), $2}'
find $R -name '*kernel_trace.csv' -delete
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_ctf_l3.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 7; }
tail -1 $R/tests.log
