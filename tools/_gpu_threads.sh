set -o pipefail
cd $GRAFT_REPO_ROOT
for t in 128 64; do
  RMD_LIBRARY=$PWD/tools/_alt/librmd_t$t.so timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/thr${t}_tests.log 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bthr_256_$i.json 2> gpurun_out/bthr_256_$i.err || exit 1
  for t in 128 64; do
    RMD_LIBRARY=$PWD/tools/_alt/librmd_t$t.so timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bthr_${t}_$i.json 2> gpurun_out/bthr_${t}_$i.err || exit 1
  done
done
# build the variants first (in this container):
#   hipcc ... -DRMD_LOOKUP_THREADS=$t -c corr_lookup.hip, linked with the other build/*.o into tools/_alt/librmd_t$t.so
