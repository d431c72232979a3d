# Round 6: w8 without ping-pong barriers and x3 with s_setprio over the MFMA phases, against the
# product: headline-only bench (w8 time, lookups) and the fp32 leg (x3), three interleaved rounds
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06j
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
AB=$PWD/tools/_ab
lib() { case $1 in product) echo $P;; *) echo $AB/librmd_$1.so;; esac; }
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off"
for round in 1 2 3; do
  for v in product w8free x3prio; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 300 python3 -u bench.py $HL > $R/b_${v}_$round.json 2> $R/b.err || { tail $R/b.err; exit 5; }
    python3 -c "
import json;d=json.loads(open('$R/b_${v}_$round.json').read().splitlines()[-1])
f=d['fp32_mode']; print('$v', round(d['value']), round(d['roofline_gemm']['avg_launch_ms'],4), round(d['roofline']['avg_launch_ms']*1e3,2), 'fp32', round(f['value']), round(f['roofline_gemm']['avg_launch_ms'],4))"
  done
done
echo done
