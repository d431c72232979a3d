# same-box A/B of the lookup over the tiles vs row fp16 pyramid layouts (tools/layout_ab.py) + counters
set -o pipefail
R=gpurun_out/layout_ab
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/layout_ab.py 30 > $R/ab.json 2> $R/ab.err || { tail -20 $R/ab.err; exit 3; }
cat $R/ab.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o run -- python3 tools/layout_ab.py 5 > /dev/null 2>> $R/ab.err || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 tools/layout_ab.py 2 > /dev/null 2>> $R/ab.err || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/sq -o run -- python3 tools/layout_ab.py 2 > /dev/null 2>> $R/ab.err || exit 6
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TD_TD_BUSY GRBM_GUI_ACTIVE --output-format csv -d $R/ta -o run -- python3 tools/layout_ab.py 2 > /dev/null 2>> $R/ab.err || exit 7
python3 tools/layout_ab_summary.py $R
