# Round-3 GPU pass: the driver's tiers (pytest -m gpu, smoke, default bench with the live PMC traffic
# passes) and a rocprofv3 kernel-trace summary of the headline step.  TAG names the outputs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/$TAG
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1; } && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 && \
timeout -k 10 500 python3 -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err && \
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --live-pmc off --fp32-mode off --model-level off --train off --hybrid off --dicl off --highres off > $O/$TAG/prof.log 2>&1
