# DAP A/B (diagnostic build): event timings + fp64 errors, then a kernel trace of the same run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-dap}
mkdir -p gpurun_out
export RMD_LIBRARY=$GRAFT_REPO_ROOT/raft-meets-dicl_amd/rmd/librmd_diag.so
timeout -k 10 200 python3 -u tools/dap_ab.py 20 > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err || exit 3
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr -o run -- python3 tools/dap_ab.py 5 > gpurun_out/${TAG}_tr.log 2>&1 || exit 4
python3 tools/trace_summary.py $(find gpurun_out/${TAG}_tr -name "*kernel_trace.csv" | head -1) dap > gpurun_out/${TAG}_trace.txt
find gpurun_out/${TAG}_tr -name "*kernel_trace.csv" -delete
echo done
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_$c -o run -- python3 tools/dap_ab.py 2 > gpurun_out/${TAG}_pmc_$c.log 2>&1 || exit 5
    python3 tools/pmc_kernel_avg.py $(find gpurun_out/${TAG}_pmc_$c -name "*counter_collection.csv" | head -1) dap > gpurun_out/${TAG}_pmc_$c.txt
    find gpurun_out/${TAG}_pmc_$c -name "*counter_collection.csv" -delete
  done
fi
echo pmc-done
