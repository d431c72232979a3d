# Round 5: S24 (24-bit) pyramid storage for the fp32 mode — parity tests, x3 GEMM and lookup times vs the
# F32 storage (fp32-f32), bench fp32 leg with live counters
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05k
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_library.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for rep in 1 2; do
  for p in fp32 fp32-f32; do
    timeout -k 10 120 python3 -u tools/x3_time.py 20 $p > $R/x3_${p}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $p $rep $(cat $R/x3_${p}_$rep.json)"
  done
  timeout -k 10 120 python3 -u tools/lookup_time.py 20 fp32 fp32-f32 bf16 > $R/lk_$rep.json 2> $R/t.err || { tail $R/t.err; exit 4; }
  echo "lookup $rep $(cat $R/lk_$rep.json)"
done
B="--steps 20 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline"
timeout -k 10 400 python3 -u bench.py $B --precision fp32 > $R/b_fp32.json 2> $R/b.err || { tail $R/b.err; exit 6; }
python3 -c "
import json;d=json.loads(open('$R/b_fp32.json').read().splitlines()[-1])
g,l=d['roofline_gemm'],d['roofline_lookup']
print('bench fp32', d['value'], 'gemm', g['avg_launch_ms'], g.get('traffic_read'), g.get('traffic_write'), g.get('mfma_busy'), 'lookup', l['avg_launch_ms'], l.get('traffic_read'), l.get('traffic_write'))"
find $R -name '*.csv' -size +4M -delete
