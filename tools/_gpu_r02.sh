# Round-2 GPU pass: parity tests, default bench line, rocprof kernel stats (+ PMC passes if PMC=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
if [ -z "$SKIPTESTS" ]; then
  timeout -k 10 ${TESTTIME:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/${TAG}_tests.log 2>&1 || exit 3
fi
if [ -z "$SKIPBENCH" ]; then
  timeout -k 10 400 python3 -u bench.py ${BENCHARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 4
fi
if [ -n "$PROF" ]; then
  R=$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}
  mkdir -p $R
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --model-level off ${BENCHARGS} > $R/bench_stats.log 2>&1 || exit 5
  find $R -name "*kernel_trace.csv" -delete                # per-dispatch traces: large; the stats stay
fi
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --model-level off > $R/fetch.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --model-level off > $R/write.log 2>&1 && \
  python3 tools/pmc_summary.py $R $R/pmc_${TAG}.json bf16 > $R/summary.log 2>&1 || exit 6
  find $R -name "*counter_collection.csv" -delete
fi
echo done
