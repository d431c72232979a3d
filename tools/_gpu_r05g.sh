# Round 5: OTF backward — product (batched G-build loads, 4-row bands, transposing unpool), all OTF tests, ablations
# (bwdabl1: no d P atomics; bwdabl2: no record-weight loads in the G build; wrong results, timing only)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05h
mkdir -p $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for v in product bwdabl1 bwdabl2; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$v -o run -- python3 tools/bench_otf.py --reps 3 --skip-4k > $R/b_$v.json 2> $R/b.err || { tail -5 $R/b.err; exit 4; }
  python3 -c "import json;d=json.load(open('$R/b_$v.json'));print('$v', {k:(round(v['otf_backward_ms'],3),round(v['volume_backward_ms'],3)) for k,v in d.items()})"
  grep -h "otf_backward_kernel\|otf_tlayout\|otf_record\|otf_unpool" $R/prof_$v/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
done
find $R -name '*kernel_trace.csv' -delete
