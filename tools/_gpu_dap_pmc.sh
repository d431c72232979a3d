# DAP D=324 counters: timing, then separate PMC passes (SQ issue/wait, MFMA busy, LDS, TA) over
# tools/dap_time.py.  Usage: bash tools/_gpu_dap_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dap}
R=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $R
timeout -k 10 120 python3 -u tools/dap_time.py 20 > $R/time.jsonl 2> $R/time.err || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $R/sq -o run -- python3 tools/dap_time.py 2 > /dev/null 2>> $R/pmc.err || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_WR TA_TA_BUSY GRBM_GUI_ACTIVE --output-format csv -d $R/lds -o run -- python3 tools/dap_time.py 2 > /dev/null 2>> $R/pmc.err || exit 5
for f in $(find $R -name '*counter_collection.csv'); do python3 tools/pmc_kernel.py $f dap_ >> $R/pmc.json; done
find $R -name '*.csv' -size +20M -delete
