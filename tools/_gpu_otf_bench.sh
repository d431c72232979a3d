# OTF vs volume timings (tools/bench_otf.py) + a kernel-trace summary of the same script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-otf_r03}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/$TAG
timeout -k 10 400 python3 -u tools/bench_otf.py --reps 5 > $O/${TAG}.json 2> $O/${TAG}.err && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 tools/bench_otf.py --reps 2 --skip-4k > $O/$TAG/prof.log 2>&1
