# Round 5: x3 MFMA-shape power check: each 32x32x16 product as two 16x16x32 MFMAs (s16t, timing only),
# with and without 24-bit level-0/1 stores (s24t), vs the product
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05d
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
lib() { if [ $1 = product ]; then echo $P; else echo $PWD/tools/_ab/librmd_$1.so; fi; }
for rep in 1 2 3; do
  for v in product s16t s24t s16s24t; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for v in s16t s16s24t; do
RMD_LIBRARY=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_$v -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 4; }
python3 tools/pmc_clock.py $R/p_$v corr_pyramid_x3 x3_$v | tee -a $R/summary.jsonl
done
find $R -name '*.csv' -size +4M -delete
