# Round 5: x3 with 24-bit level-0/1 stores (timing variant, s24t) vs the product; zero operands (power check)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05c
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
lib() { if [ $1 = product ]; then echo $P; else echo $PWD/tools/_ab/librmd_$1.so; fi; }
for rep in 1 2 3; do
  for v in product s24t; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
  X3_FILL=zero timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_zero_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
  echo "x3 zero-operands $rep $(cat $R/t_zero_$rep.json)"
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
RMD_LIBRARY=$(lib s24t) timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_s24t -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 4; }
python3 tools/pmc_clock.py $R/p_s24t corr_pyramid_x3 x3_s24t | tee -a $R/summary.jsonl
X3_FILL=zero timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_zero -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 4; }
python3 tools/pmc_clock.py $R/p_zero corr_pyramid_x3 x3_zero_operands | tee -a $R/summary.jsonl
find $R -name '*.csv' -size +4M -delete
