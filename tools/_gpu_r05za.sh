# Round 5: G build diagnostics — build alone (12 lookups / 0 lookups / round-4 sequential path) and
# counters of the build kernel
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${1:-r05za}
mkdir -p $R
timeout -k 10 120 python3 -u tools/bench_grad_build.py 20 > $R/gb.jsonl 2> $R/gb.err || { tail -5 $R/gb.err; exit 2; }
cat $R/gb.jsonl
i=0
for P in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU GRBM_GUI_ACTIVE" "TA_TA_BUSY TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/p$i -o run -- python3 tools/bench_grad_build.py 2 > /dev/null 2> $R/p$i.err || { tail -5 $R/p$i.err; exit 4; }
  python3 tools/pmc_kernel.py $R/p$i/run_counter_collection.csv corr_grad_build > $R/p$i.json
  cat $R/p$i.json
done
find $R -name '*.csv' -size +4M -delete
