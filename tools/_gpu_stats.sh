set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/stats
mkdir -p $R
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 ${SCRIPT:-bench.py} ${ARGS:---steps 10 --warmup 2 --no-cpu-baseline} > $R/run.log 2>&1
