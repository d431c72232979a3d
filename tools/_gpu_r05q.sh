# Round 5: level-3 chunks 1x4 in every layout (product) vs 1x2 (l3x2 = the previous build) — parity tests
# of every GEMM path, then the bench step's lookup in bf16 (tiles), fp32 (S24 rows) and fp32-f32 (F32 rows)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05q
mkdir -p $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_corr.py tests/test_library.py tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
B="--steps 30 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off --event-every 1"
for rep in 1 2 3; do
  for v in product l3x2; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    for p in bf16 fp32 fp32-f32; do
      RMD_LIBRARY=$L timeout -k 10 200 python3 -u bench.py $B --precision $p > $R/b_${v}_${p}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 3; }
      python3 -c "
import json;d=json.loads(open('$R/b_${v}_${p}_$rep.json').read().splitlines()[-1])
print('bench $v $p $rep', round(d['value'],1), round(d['ms_per_step'],4), 'gemm', round(d['roofline_gemm']['avg_launch_ms'],4), 'lookup', round(d['roofline_lookup']['avg_launch_ms']*1e3,2))"
    done
  done
done
