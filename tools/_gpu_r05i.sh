# Round 5: OTF backward (fixed-point d P, batched G build, transposing unpool) and the RAFT volume backward
# with bf16-mode grad GEMMs — GPU OTF + corr tests, timings, kernel stats, ablations
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05i
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_otf.py tests/test_gpu_corr.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for v in product bwdabl1 bwdabl2; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$v -o run -- python3 tools/bench_otf.py --reps 3 --skip-4k > $R/b_$v.json 2> $R/b.err || { tail -5 $R/b.err; exit 4; }
  python3 -c "import json;d=json.load(open('$R/b_$v.json'));print('$v', {k:(round(v['otf_backward_ms'],3),round(v['volume_backward_ms'],3)) for k,v in d.items()})"
done
for p in bf16 fp32; do
  timeout -k 10 200 python3 -u tools/bench_corr_bwd.py 10 $p cfg2 > $R/corr_bwd_$p.json 2> $R/cb.err || { tail -5 $R/cb.err; exit 5; }
  python3 -c "import json;d=json.load(open('$R/corr_bwd_$p.json'));print('corr_bwd $p', {k:d[k] for k in d if 'ms' in k})"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_cb -o run -- python3 tools/bench_corr_bwd.py 5 bf16 cfg2 > /dev/null 2> $R/cb.err || { tail -5 $R/cb.err; exit 6; }
find $R -name '*kernel_trace.csv' -delete
