# Round 5: SQ counters + effective clock of the x3 GEMM (product and stores-dropped build) and of w8
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05a
mkdir -p $R
rocprofv3 -L > $R/counters.txt 2>&1 || true
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
A=$PWD/tools/_ab/librmd_x3abl1.so
for v in product x3abl1; do
  L=$P; [ $v = x3abl1 ] && L=$A
  RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_$v.json 2> $R/t.err || { tail $R/t.err; exit 3; }
  echo "time $v $(cat $R/t_$v.json)"
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for v in product x3abl1; do
  L=$P; [ $v = x3abl1 ] && L=$A
  for pass in A B; do
    C=$SQA; [ $pass = B ] && C=$SQB
    RMD_LIBRARY=$L timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/p_${v}_$pass -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_${v}_$pass.err || { tail -5 $R/p_${v}_$pass.err; exit 4; }
    python3 tools/pmc_clock.py $R/p_${v}_$pass corr_pyramid_x3 x3_${v}_$pass | tee -a $R/summary.jsonl
  done
done
for pass in A B; do
  C=$SQA; [ $pass = B ] && C=$SQB
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/p_w8_$pass -o run -- python3 tools/x3_time.py 6 bf16 > /dev/null 2> $R/p_w8_$pass.err || { tail -5 $R/p_w8_$pass.err; exit 5; }
  python3 tools/pmc_clock.py $R/p_w8_$pass corr_pyramid_w8 w8_$pass | tee -a $R/summary.jsonl
done
find $R -name '*.csv' -size +4M -delete
