# Round-3 pass on the merged-level OTF tree: OTF A/B, full GPU suite, smoke, bench
set -o pipefail
export TMPDIR=/tmp
PRECS=bf16 VARIANTS="otf_old otf_b12ql otf_b14ql otf_b14qln512 otf_b12qln512 otf_b11n512" bash tools/_gpu_r03k.sh || exit 2
cp gpurun_out/r03k/otf_ab.jsonl gpurun_out/r03k/otf_ab_b.jsonl
PRECS=fp32 VARIANTS="otf_old otf_x12ql" bash tools/_gpu_r03k.sh || exit 3
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 4; }
tail -1 gpurun_out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_r03l.json 2> gpurun_out/bench_r03l.err || exit 6
echo done
