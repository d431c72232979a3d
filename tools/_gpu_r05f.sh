# Round 5: OTF backward rewrite (multi-row bands, owner-thread G build, fixed-point d P) — GPU OTF tests,
# then cfg2 b8 training timings vs the round-4 kernel (tools/_ab/librmd_otfr04.so)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05f
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -3 $R/tests.log
for rep in 1 2; do
  for v in product otfr04; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 300 python3 -u tools/bench_otf.py --reps 5 --skip-4k > $R/b_${v}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 3; }
    python3 -c "import json;d=json.load(open('$R/b_${v}_$rep.json'));print('$v $rep', {k:(round(v['otf_backward_ms'],3),round(v['volume_backward_ms'],3),round(v['otf_forward_ms'],3)) for k,v in d.items()})"
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_otf.py --reps 3 --skip-4k > /dev/null 2> $R/prof.err || { tail -5 $R/prof.err; exit 4; }
grep -h "otf_\|corr_lookup_backward\|grad_gemm" $R/prof/*kernel_stats.csv | cut -c1-150
find $R -name '*kernel_trace.csv' -delete
