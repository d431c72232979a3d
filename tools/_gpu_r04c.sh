# Round-4 lookup counters: SQ instruction / wait / issue counters of the product lookup and the
# no-traffic build (abl3), one rocprofv3 --pmc pass per counter group, each under its own KILL timeout
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04c
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
A=$PWD/tools/_ab/librmd_abl3.so
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL"
G3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"
G4="TA_BUSY_avr TA_TA_BUSY_sum"
n=0
for lib in $P $A; do
  for g in "$G1" "$G2" "$G3"; do
    n=$((n+1))
    RMD_LIBRARY=$lib timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d $R/p$n -o run -- python3 tools/lookup_time.py 3 bf16 > $R/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $R/p$n.log; exit 2; }
    f=$(find $R/p$n -name '*counter_collection.csv' | head -1)
    echo "== pass $n $(basename $lib)"
    python3 tools/pmc_kernel.py $f corr_lookup_kernel
  done
done
