# Round 5: x3 one-wave-per-SIMD variants (v2: QT query tiles per pass) vs the product; lookup grid order A/B
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05b
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
lib() { if [ $1 = product ]; then echo $P; else echo $PWD/tools/_ab/librmd_$1.so; fi; }
for rep in 1 2; do
  for v in product v2q2 v2q1 v2q2d8 v2q2abl1; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "x3 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for v in v2q2 v2q1; do
  RMD_LIBRARY=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $R/p_$v -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_$v.err || { tail -5 $R/p_$v.err; exit 4; }
  python3 tools/pmc_clock.py $R/p_$v corr_pyramid_x3 x3_$v | tee -a $R/summary.jsonl
done
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/p_tcc -o run -- python3 tools/x3_time.py 6 fp32 > /dev/null 2> $R/p_tcc.err || { tail -5 $R/p_tcc.err; exit 5; }
python3 tools/pmc_clock.py $R/p_tcc corr_pyramid_x3 x3_product_tcc | tee -a $R/summary.jsonl
B="--steps 20 --warmup 10 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --no-cpu-baseline --live-pmc off"
for rep in 1 2; do
  for v in product lkz1 lkz2; do
    RMD_LIBRARY=$(lib $v) timeout -k 10 200 python3 -u bench.py $B > $R/b_${v}_$rep.json 2> $R/b.err || { tail $R/b.err; exit 6; }
    python3 -c "import json;d=json.loads(open('$R/b_${v}_$rep.json').read().splitlines()[-1]);print('lookup $v $rep', d['value'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])"
  done
done
find $R -name '*.csv' -size +4M -delete
