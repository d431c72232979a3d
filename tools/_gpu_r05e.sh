# Round 5: the 16x16x32 x3 GEMM (product) — correctness (GPU corr / e2e / ctf-l3 tests) and A/B vs the
# 32x32x16 form (-DRMD_X3_SHAPE=32)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05e
mkdir -p $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -3 $R/tests.log
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
lib() { if [ $1 = product ]; then echo $P; else echo $PWD/tools/_ab/librmd_$1.so; fi; }
for rep in 1 2 3; do
  for v in product x3s32; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_x3s -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p.err || { tail -5 $R/p.err; exit 4; }
python3 tools/pmc_clock.py $R/p_x3s corr_pyramid_x3 x3s_product | tee -a $R/summary.jsonl
find $R -name '*.csv' -size +4M -delete
