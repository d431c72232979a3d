# Round-3 final pass (final tree): full GPU suite, smoke, bench line, rocprofv3 kernel stats of the bench, OTF timing
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r03n
mkdir -p $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -20 $R/tests.log; exit 2; }
tail -1 $R/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit 3
timeout -k 10 300 python3 -u bench.py > $R/bench.json 2> $R/bench.err || exit 4
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/prof.log 2>&1 || exit 5
timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/otf_time.json 2> $R/otf_time.err || exit 6
find $R -name '*.csv' -size +20M -delete
PRECS=bf16 VARIANTS="otf_b12qln512 otf_b11ql otf_b11qln512 otf_b14qln512" bash tools/_gpu_r03k.sh > $R/ab.log 2>&1 || exit 7
echo done
