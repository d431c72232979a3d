# round 3: tiles-layout pyramid (w8) + lookup — GPU tests of the correlation path, then a short bench
set -o pipefail
R=gpurun_out/r03b
mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_graph.py tests/test_library.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 3; }
tail -3 $R/tests.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --model-level off --fp32-mode off \
  --train off --hybrid off --dicl off --highres off > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 4; }
cat $R/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print({k:d[k] for k in ('roofline','roofline_gemm')})"
