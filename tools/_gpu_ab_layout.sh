set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_new_$i.json 2>/dev/null || exit 1
  RMD_LIBRARY=$GRAFT_REPO_ROOT/tools/_bin/librmd_rowchunk.so timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_old_$i.json 2>/dev/null || exit 1
done
RMD_ABLATE=1 timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_new_nostore.json 2>/dev/null
