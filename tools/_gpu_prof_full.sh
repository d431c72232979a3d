# Full measurement pass: bench kernel stats + FETCH/WRITE PMC passes + bench line + component kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/prof
C=$GRAFT_REPO_ROOT/gpurun_out/comp
mkdir -p $R $C
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/bench_stats.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/write.log 2>&1 && \
python3 tools/pmc_summary.py $R profiles/pmc_r01.json bf16 > $R/summary.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && \
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $C -o run -- python3 tools/bench_components.py 10 heads > $C/comp.json 2> $C/comp.err
