# Two slot blocks per lookup wave (RMD_LOOKUP_TWO, occupancy 5 / 6) vs the product: bitwise output
# digests, the corr parity tests on the variant, per-position lookup times in the bench step, and the
# headline-only bench line; two interleaved rounds
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06q}
mkdir -p $R
for v in prod two5 two6; do
  if [ $v = prod ]; then L=raft-meets-dicl_amd/rmd/librmd.so; else L=tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -k 10 120 python3 tools/lookup_outputs_sha.py 2>/dev/null | tee -a $R/summary.txt || exit 2
done
RMD_LIBRARY=tools/_ab/librmd_two5.so timeout -k 10 600 python -u -m pytest tests/test_gpu_corr.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests_two5.log 2>&1 || { tail -20 $R/tests_two5.log; exit 3; }
tail -1 $R/tests_two5.log | tee -a $R/summary.txt
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off --fp32-mode off"
for round in 1 2; do
for v in prod two5 two6; do
  if [ $v = prod ]; then L=raft-meets-dicl_amd/rmd/librmd.so; else L=tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L LOOKUP_CONTEXT_MODES=bench,samecoord timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv \
    -d $R/ctx_${v}_$round -o run -- python3 tools/lookup_context.py 10 > $R/ctx_${v}_$round.out 2>&1 || { tail $R/ctx_${v}_$round.out; exit 4; }
  f=$(ls $R/ctx_${v}_$round/*kernel_trace.csv $R/ctx_${v}_$round/*/*kernel_trace.csv 2>/dev/null | head -1)
  echo "ctx $v $round $(LOOKUP_CONTEXT_MODES=bench,samecoord python3 tools/lookup_context.py --summary $f)" | tee -a $R/summary.txt
  RMD_LIBRARY=$L timeout -k 10 300 python3 bench.py $HL --steps 30 --warmup 5 > $R/hl_${v}_$round.json 2> $R/hl_${v}_$round.err || { tail $R/hl_${v}_$round.err; exit 5; }
  python3 -c "
import json;d=json.loads(open('$R/hl_${v}_$round.json').read().splitlines()[-1])
print('hl $v $round', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms']*1e3,2), round(d['roofline']['frac'],3), round(d['roofline_gemm']['avg_launch_ms']*1e3,1))" | tee -a $R/summary.txt
done
done
echo done
