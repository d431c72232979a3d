# Round 5: fp32-mode step with S24 (fp32) vs F32 (fp32-f32) pyramid storage in bench.py's cold-read
# context (GEMM then 12 lookups), alternating; OTF lookup time vs batch (grid depth: 896 / 1792 / 2688 blocks)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05o
mkdir -p $R
B="--steps 30 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off --event-every 1"
for rep in 1 2 3; do
  for p in fp32 fp32-f32; do
    timeout -k 10 200 python3 -u bench.py $B --precision $p > $R/b_${p}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 3; }
    python3 -c "
import json;d=json.loads(open('$R/b_${p}_$rep.json').read().splitlines()[-1])
print('bench $p $rep', round(d['value'],1), round(d['ms_per_step'],4), 'gemm', round(d['roofline_gemm']['avg_launch_ms'],4), 'lookup', round(d['roofline_lookup']['avg_launch_ms']*1e3,2))"
  done
done
for bb in 4 8 12; do
  OTF_SHAPE=$bb,55,128 timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 > $R/otf_b$bb.json 2> $R/t.err || { tail $R/t.err; exit 4; }
  echo "otf b$bb $(cat $R/otf_b$bb.json)"
done
