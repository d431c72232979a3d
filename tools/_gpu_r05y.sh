# Round 5: RAFT lookup backward with every load outside branches (clamped tap rows / chunk rows /
# chunks, all pieces of a row loaded before its updates) = product vs the previous kernel (bwdold);
# parity tests first, then the cfg2 b8 backward in both methodologies
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05y
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for rep in 1 2; do
  for v in product bwdold; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    for p in bf16 fp32; do
      RMD_LIBRARY=$L timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 $p cfg2 > $R/cb_${v}_${p}_$rep.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
      python3 -c "import json;d=json.load(open('$R/cb_${v}_${p}_$rep.json'));print('corr_bwd $v $p $rep', {k:round(d[k],3) for k in d if 'ms' in k})"
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 6; }
grep -h "corr_lookup_backward\|grad_gemm" $R/prof/run_kernel_stats.csv | cut -c1-160
find $R -name '*kernel_trace.csv' -delete
