# OTF lookup SQ counters (diag build) under ablation modes: where does the non-MFMA, non-store time go?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so
R=gpurun_out/otfpmc
mkdir -p $R
for A in 0 3; do
  RMD_OTF_ABLATE=$A timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $R/a${A}_a -o run -- python3 tools/otf_probe.py 4 bf16 > $R/a${A}_a.log 2>&1 || exit 3
  RMD_OTF_ABLATE=$A timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $R/a${A}_b -o run -- python3 tools/otf_probe.py 4 bf16 > $R/a${A}_b.log 2>&1 || exit 4
  for p in a b; do
    python3 tools/pmc_kernel_avg.py $(find $R/a${A}_$p -name "*counter_collection.csv" | head -1) otf_lookup > $R/a${A}_$p.txt
    find $R/a${A}_$p -name "*counter_collection.csv" -delete
  done
done
echo done
