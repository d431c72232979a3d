set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for s in 3 2 5 9; do
    RMD_LOOKUP_SPLIT=$s timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bsplit_${s}_$i.json 2> gpurun_out/bsplit_${s}_$i.err || exit 1
  done
done
