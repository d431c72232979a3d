# Round 5: S24 with 1x4 level-3 chunks — parity tests; fp32-mode bench step (cold lookups after the GEMM):
# S24 (fp32-s24) vs F32 (fp32-f32) storage, and S24 with 16+8-byte level-0/1 chunk loads (s24ld)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05p
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_library.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
B="--steps 30 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off --event-every 1"
for rep in 1 2 3; do
  for v in s24 f32 s24ld; do
    case $v in s24) L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; p=fp32-s24;; f32) L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; p=fp32-f32;; s24ld) L=$PWD/tools/_ab/librmd_s24ld.so; p=fp32-s24;; esac
    RMD_LIBRARY=$L timeout -k 10 200 python3 -u bench.py $B --precision $p > $R/b_${v}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 3; }
    python3 -c "
import json;d=json.loads(open('$R/b_${v}_$rep.json').read().splitlines()[-1])
print('bench $v $rep', round(d['value'],1), round(d['ms_per_step'],4), 'gemm', round(d['roofline_gemm']['avg_launch_ms'],4), 'lookup', round(d['roofline_lookup']['avg_launch_ms']*1e3,2))"
  done
done
