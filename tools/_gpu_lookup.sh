# lookup parity tests (product library) then the A/B of lookup variants (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-lk}
mkdir -p gpurun_out
if [ -z "$SKIPTESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_corr.py} > gpurun_out/${TAG}_tests.log 2>&1 || exit 3
fi
RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so RMD_AB=${AB:-XCH=1,XCH=0} timeout -k 10 300 python3 -u tools/lookup_ab.py 20 bf16 > gpurun_out/${TAG}_ab_bf16.json 2> gpurun_out/${TAG}_ab_bf16.err || exit 4
RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so RMD_AB=${AB:-XCH=1,XCH=0} timeout -k 10 300 python3 -u tools/lookup_ab.py 10 fp32 > gpurun_out/${TAG}_ab_fp32.json 2> gpurun_out/${TAG}_ab_fp32.err || exit 5
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python3 -u bench.py ${BENCHARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 6
fi
echo done
