# Lookup pyramid-load cache policy A/B (RMD_LOOKUP_LAUX: 0 product, 1 sc0, 2 nt, 16 sc1, 18 sc1+nt):
# per-position lookup times in the bench step (tools/lookup_context.py, bench + samecoord modes) and
# the headline-only bench line per library, two interleaved rounds
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06o}
mkdir -p $R
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off"
for round in 1 2; do
for v in prod laux2 laux1 laux16 laux18; do
  if [ $v = prod ]; then L=raft-meets-dicl_amd/rmd/librmd.so; else L=tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L LOOKUP_CONTEXT_MODES=bench,samecoord timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv \
    -d $R/ctx_${v}_$round -o run -- python3 tools/lookup_context.py 10 > $R/ctx_${v}_$round.out 2>&1 || { tail $R/ctx_${v}_$round.out; exit 2; }
  f=$(ls $R/ctx_${v}_$round/*kernel_trace.csv $R/ctx_${v}_$round/*/*kernel_trace.csv 2>/dev/null | head -1)
  echo "ctx $v $round $(LOOKUP_CONTEXT_MODES=bench,samecoord python3 tools/lookup_context.py --summary $f)" | tee -a $R/summary.txt
  RMD_LIBRARY=$L timeout -k 10 300 python3 bench.py $HL --steps 30 --warmup 5 > $R/hl_${v}_$round.json 2> $R/hl_${v}_$round.err || { tail $R/hl_${v}_$round.err; exit 3; }
  python3 -c "
import json;d=json.loads(open('$R/hl_${v}_$round.json').read().splitlines()[-1])
print('hl $v $round', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms']*1e3,2), round(d['roofline_gemm']['avg_launch_ms']*1e3,1), 'fp32', round(d['fp32_mode']['value']), round(d['fp32_mode']['roofline_lookup']['avg_launch_ms']*1e3,2))" | tee -a $R/summary.txt
done
done
echo done
