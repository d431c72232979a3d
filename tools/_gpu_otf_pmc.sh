# OTF lookup counters at cfg2 bf16: SQ issue / wait / MFMA busy, LDS and TA, one pass each over
# tools/otf_time.py.  Usage: bash tools/_gpu_otf_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-otf}
R=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $R
timeout -k 10 120 python3 -u tools/otf_time.py 5 bf16 > $R/time.json 2> $R/time.err || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $R/sq -o run -- python3 tools/otf_time.py 1 bf16 > /dev/null 2>> $R/pmc.err || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR TA_TA_BUSY --output-format csv -d $R/lds -o run -- python3 tools/otf_time.py 1 bf16 > /dev/null 2>> $R/pmc.err || exit 5
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAVES SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $R/mem -o run -- python3 tools/otf_time.py 1 bf16 > /dev/null 2>> $R/pmc.err || true
for f in $(find $R -name '*counter_collection.csv'); do python3 tools/pmc_kernel.py $f otf_lookup >> $R/pmc.json; done
find $R -name '*.csv' -size +20M -delete
