# SQ / TA counter passes of the lookup kernel for each variant in VARIANTS (diag build, lookup_ab.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so
R=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmclk}
mkdir -p $R
for V in ${VARIANTS:-V=2 V=3}; do
  export RMD_AB=$V
  n=$(echo $V | tr '=+' '__')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/${n}_a -o run -- python3 tools/lookup_ab.py 2 bf16 > $R/${n}_a.log 2>&1 || exit 5
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d $R/${n}_b -o run -- python3 tools/lookup_ab.py 2 bf16 > $R/${n}_b.log 2>&1 || exit 6
  for p in a b; do f=$(find $R/${n}_$p -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernel.py $f corr_lookup > $R/${n}_$p.json; rm -f $f; done
done
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY TD_TD_BUSY GRBM_GUI_ACTIVE --output-format csv -d $R/ta -o run -- python3 tools/lookup_ab.py 2 bf16 > $R/ta.log 2>&1 || exit 7
f=$(find $R/ta -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernel.py $f corr_lookup > $R/ta.json; rm -f $f
echo done
