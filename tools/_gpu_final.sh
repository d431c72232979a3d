# Round-end rehearsal: the driver's GPU tiers (pytest -m gpu, smoke, bench) plus the measurement pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && \
bash tools/_gpu_prof_full.sh && \
timeout -k 10 300 python3 -u tools/bench_components.py 20 > gpurun_out/components.json 2> gpurun_out/components.err
