# Round 6: x3s (fp32-mode GEMM) counters and ablations on the product form; w8 per-level store policy A/B
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06a
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
AB=$PWD/tools/_ab
lib() { case $1 in product) echo $P;; *) echo $AB/librmd_$1.so;; esac; }
for round in 1 2; do
  for v in product x3abl1 x3abl2 x3abl3; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 30 fp32 > $R/t_${v}_$round.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "time $v $(cat $R/t_${v}_$round.json)"
  done
  X3_FILL=zero timeout -k 10 120 python3 -u tools/x3_time.py 30 fp32 > $R/t_zero_$round.json 2> $R/t.err || { tail $R/t.err; exit 3; }
  echo "time zero $(cat $R/t_zero_$round.json)"
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
SQC="SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_WAIT_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_IFETCH GRBM_GUI_ACTIVE"
for v in product x3abl2 x3abl3; do
  for pass in A B C; do
    eval C=\$SQ$pass
    RMD_LIBRARY=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/p_${v}_$pass -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_${v}_$pass.err || { tail -5 $R/p_${v}_$pass.err; echo "pmc $v $pass failed"; continue; }
    python3 tools/pmc_clock.py $R/p_${v}_$pass corr_pyramid_x3 x3_${v}_$pass | tee -a $R/summary.jsonl
  done
done
HL="--no-cpu-baseline --model-level off --fp32-mode off --live-pmc off --train off --hybrid off --dicl off --highres off"
for round in 1 2; do
  for v in product w8auxh0; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 200 python3 -u bench.py $HL > $R/b_${v}_$round.json 2> $R/b.err || { tail $R/b.err; exit 5; }
    python3 -c "
import json;d=json.loads(open('$R/b_${v}_$round.json').read().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])"
  done
done
for v in product w8auxh0; do
  LOOKUP_CONTEXT_MODES=bench,nogemm RMD_LIBRARY=$(lib $v) timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/lc_$v -o run -- python3 tools/lookup_context.py 20 > /dev/null 2> $R/lc_$v.err || { tail -5 $R/lc_$v.err; exit 6; }
  echo "ctx $v $(LOOKUP_CONTEXT_MODES=bench,nogemm python3 tools/lookup_context.py --summary $(python3 -c "import glob;print(glob.glob('$R/lc_$v/**/*kernel_trace.csv',recursive=True)[0])"))"
done
find $R -name '*.csv' -size +4M -delete
echo done
