# PMC passes (one rocprofv3 run per counter group) of tools/gemm_ab.py for the RMD_AB variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p $R
export RMD_AB_ROUNDS=1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/a -o run -- python3 ${CMD:-tools/gemm_ab.py 5} > $R/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $R/b -o run -- python3 ${CMD:-tools/gemm_ab.py 5} > $R/b.log 2>&1 || exit 5
for p in a b; do f=$(find $R/$p -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernel.py $f ${PAT:-corr_pyramid_w8} > $R/$p.json; done
echo done
