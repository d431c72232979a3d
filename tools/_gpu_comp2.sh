# Component timings (HIP events) and a rocprofv3 kernel trace of the same script (per-kernel medians).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-comp2}
R=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $R
timeout -k 10 400 python3 -u tools/bench_components.py 20 > $R/components.json 2> $R/components.err || exit 3
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 tools/bench_components.py 5 > $R/prof.log 2>&1 || exit 4
python3 tools/trace_summary.py $(find $R/prof -name "*kernel_trace.csv" | head -1) rmd > $R/kernels.txt
find $R -name "*kernel_trace.csv" -delete
echo done
