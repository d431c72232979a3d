# Round 5: S24 in the tiles layout (x3 prep in tiles slot order, 2x4 level-0/1 chunks) — parity tests of
# every GEMM path, then the fp32-mode bench step: S24 tiles (product) vs S24 rows (s24rows = previous build)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05t
mkdir -p $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_corr.py tests/test_library.py tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
B="--steps 30 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off --event-every 1"
for rep in 1 2 3; do
  for v in product s24rows; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 200 python3 -u bench.py $B --precision fp32 > $R/b_${v}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 3; }
    python3 -c "
import json;d=json.loads(open('$R/b_${v}_$rep.json').read().splitlines()[-1])
print('bench $v $rep', round(d['value'],1), round(d['ms_per_step'],4), 'gemm', round(d['roofline_gemm']['avg_launch_ms'],4), 'lookup', round(d['roofline_lookup']['avg_launch_ms']*1e3,2))"
  done
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --precision fp32 > $R/b_pmc.json 2> $R/b.err || { tail $R/b.err; exit 4; }
python3 -c "
import json;d=json.loads(open('$R/b_pmc.json').read().splitlines()[-1]);g,l=d['roofline_gemm'],d['roofline_lookup']
print('pmc', d['value'], 'gemm', g['avg_launch_ms'], g.get('traffic_write'), g.get('mfma_busy'), 'lookup', l['avg_launch_ms'], l.get('traffic_read'), l.get('traffic_write'))"
