# Round 5: x3 MFMA issue order — product (three dependent products per accumulator back to back) vs ord1
# (product outer: 8 independent accumulators between dependent MFMAs); bitwise-equal checksums expected
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05r
mkdir -p $R
for rep in 1 2 3; do
  for v in product ord1; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in product ord1; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_$v -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_$v.err || { tail -5 $R/p_$v.err; exit 4; }
  python3 tools/pmc_clock.py $R/p_$v corr_pyramid_x3 x3_$v | tee -a $R/summary.jsonl
done
find $R -name '*.csv' -size +4M -delete
