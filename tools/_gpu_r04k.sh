# Round-4: SQ counters of the OTF lookup (cfg2 bf16), one rocprofv3 --pmc pass per counter group
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04k
mkdir -p $R
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS"
G3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
G4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
n=0
for g in "$G1" "$G2" "$G3" "$G4"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d $R/p$n -o run -- python3 tools/otf_time.py 3 bf16 > $R/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $R/p$n.log; exit 2; }
  f=$(find $R/p$n -name '*counter_collection.csv' | head -1)
  echo "== pass $n"; python3 tools/pmc_kernel.py $f otf_lookup_kernel
done
