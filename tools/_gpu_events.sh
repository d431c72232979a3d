set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for e in 1 5 1000; do
    timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --event-every $e > gpurun_out/bev_${e}_$i.json 2> gpurun_out/bev_${e}_$i.err || exit 1
  done
done
timeout -k 10 200 python -u tools/graph_step_ab.py 5 > gpurun_out/graph_ab2.json 2> gpurun_out/graph_ab2.err
