# DICL stack backward A/B (diagnostic build): event timings + kernel trace medians
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RMD_LIBRARY=$GRAFT_REPO_ROOT/raft-meets-dicl_amd/rmd/librmd_diag.so
R=gpurun_out/diclbwd
mkdir -p $R
timeout -k 10 300 python3 -u tools/dicl_bwd_ab.py 10 > $R/ab.json 2> $R/ab.err || exit 3
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $R/tr -o run -- python3 tools/dicl_bwd_ab.py 3 > $R/tr.log 2>&1 || exit 4
python3 tools/trace_summary.py $(find $R/tr -name "*kernel_trace.csv" | head -1) backward > $R/trace.txt
find $R/tr -name "*kernel_trace.csv" -delete
echo done
