# Round 6: x3 GEMM without ping-pong barriers (free-running waves) vs the product; ablations on the
# round-6 epilogue; x3_time back to back and the headline-only bench's fp32 leg per library
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06g
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
AB=$PWD/tools/_ab
lib() { case $1 in product) echo $P;; *) echo $AB/librmd_$1.so;; esac; }
for round in 1 2 3; do
  for v in product free abl2 abl3 nobal; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 30 fp32 > $R/t_${v}_$round.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "time $v $(cat $R/t_${v}_$round.json)"
  done
done
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off"
for round in 1 2; do
  for v in product free; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 300 python3 -u bench.py $HL > $R/b_${v}_$round.json 2> $R/b.err || { tail $R/b.err; exit 5; }
    python3 -c "
import json;d=json.loads(open('$R/b_${v}_$round.json').read().splitlines()[-1])
f=d['fp32_mode']; print('$v', d['value'], 'fp32', f['value'], f['roofline_gemm']['avg_launch_ms'])"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for v in free abl2 abl3; do
  RMD_LIBRARY=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_${v} -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_${v}.err || { tail -5 $R/p_${v}.err; exit 4; }
  python3 tools/pmc_clock.py $R/p_${v} corr_pyramid_x3 x3_${v}_A | tee -a $R/summary.jsonl
done
find $R -name '*.csv' -size +4M -delete
echo done
