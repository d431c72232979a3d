# Round 5: G build (rmd_corr_grad_build: all lookups of a forward in one pass that writes G once)
# vs the round-4 path (zero fill + one rmd_corr_lookup_backward per lookup); parity first
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${1:-r05z}
mkdir -p $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_grad_build.py -m gpu -x -v --timeout 120 --timeout-method thread > $R/tests_build.log 2>&1 || { tail -40 $R/tests_build.log; exit 2; }
tail -3 $R/tests_build.log
for rep in 1 2; do
  for gb in 1 0; do
    for p in bf16 fp32; do
      RMD_GRAD_BUILD=$gb timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 $p cfg2 > $R/cb_gb${gb}_${p}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
      python3 -c "import json;d=json.load(open('$R/cb_gb${gb}_${p}_$rep.json'));print('corr_bwd build=$gb $p $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
grep -h "grad_build\|lookup_backward\|grad_gemm\|FillFunctor" $R/prof/run_kernel_stats.csv | cut -c1-160
find $R -name '*kernel_trace.csv' -delete
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_ctf_l3.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 7; }
tail -2 $R/tests.log
