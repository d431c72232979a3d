# Lookup occupancy A/B: product librmd.so (waves_per_eu 8) vs librmd_wpe1.so (no occupancy hint, SGPRs cap it at 7),
# bench lines interleaved, then kernel-trace medians of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/wpe
mkdir -p $R
A="--steps 50 --warmup 10 --no-cpu-baseline --model-level off --train off --hybrid off --dicl off --event-every 1"
for i in 1 2 3; do
  for L in librmd librmd_wpe1; do
    RMD_LIBRARY=raft-meets-dicl_amd/rmd/$L.so timeout -k 10 200 python3 -u bench.py $A > $R/${L}_$i.json 2> $R/${L}_$i.err || exit 3
    echo "$L $i done"
  done
done
for L in librmd librmd_wpe1; do
  RMD_LIBRARY=raft-meets-dicl_amd/rmd/$L.so timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $R/tr_$L -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --model-level off --train off --hybrid off --dicl off > $R/tr_$L.log 2>&1 || exit 4
  python3 tools/trace_summary.py $(find $R/tr_$L -name '*kernel_trace.csv') corr_lookup > $R/tr_$L.txt
  find $R/tr_$L -name '*kernel_trace.csv' -delete
done
echo done
