# Round 6: GPU tests for the S24 epilogue rewrite, the tightened fp32 gates, the OTF bound fix, the
# pending-gradient flush, DDP at world 4; x3 GEMM A/B (r05 epilogue vs round-6 epilogue) + counters
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06b
mkdir -p $R
timeout -k 10 120 python3 -u tools/s24_debug.py 2 32 24 40 > $R/s24.txt 2>&1 || { tail -30 $R/s24.txt; exit 1; }
cat $R/s24.txt
timeout -k 10 120 python3 -u tools/s24_debug.py 8 256 55 128 > $R/s24b.txt 2>&1 || { tail -30 $R/s24b.txt; exit 1; }
cat $R/s24b.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_otf.py tests/test_gpu_grad_build.py tests/test_distributed.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -3 $R/tests.log
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
AB=$PWD/tools/_ab
lib() { case $1 in product) echo $P;; *) echo $AB/librmd_$1.so;; esac; }
for round in 1 2 3; do
  for v in r05 nobal product; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 30 fp32 > $R/t_${v}_$round.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "time $v $(cat $R/t_${v}_$round.json)"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for v in product; do
  for pass in A B; do
    eval C=\$SQ$pass
    RMD_LIBRARY=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/p_${v}_$pass -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_${v}_$pass.err || { tail -5 $R/p_${v}_$pass.err; exit 4; }
    python3 tools/pmc_clock.py $R/p_${v}_$pass corr_pyramid_x3 x3_${v}_$pass | tee -a $R/summary.jsonl
  done
done
HL="--no-cpu-baseline --model-level off --live-pmc off --train off --hybrid off --dicl off --highres off"
timeout -k 10 300 python3 -u bench.py $HL > $R/b.json 2> $R/b.err || { tail $R/b.err; exit 5; }
python3 -c "
import json;d=json.loads(open('$R/b.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gemm']['avg_launch_ms'])
f=d['fp32_mode']; print('fp32', f['value'], f['ms_per_step'], f['roofline_gemm']['avg_launch_ms'], f['roofline_lookup']['avg_launch_ms'])"
find $R -name '*.csv' -size +4M -delete
echo done
