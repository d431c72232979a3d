# Round 5: G build ablation (no grad_out traffic) and instruction-mix counters of the product build kernel
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05zf
mkdir -p $R
for v in product abl1; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/bench_grad_build.py 20 > $R/gb_$v.jsonl 2> $R/gb.err || { tail -5 $R/gb.err; exit 3; }
  echo "== $v"; head -1 $R/gb_$v.jsonl
done
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/p$i -o run -- python3 tools/bench_grad_build.py 2 > /dev/null 2> $R/p$i.err || { tail -5 $R/p$i.err; exit 4; }
  python3 tools/pmc_kernel.py $R/p$i/run_counter_collection.csv corr_grad_build > $R/p$i.json
  cat $R/p$i.json
done
find $R -name '*.csv' -size +4M -delete
