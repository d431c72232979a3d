# A/B timing run (diagnostic build): GEMM variants named in RMD_AB, then the product bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/gemm_ab.py 20 > gpurun_out/${TAG}_gemm_ab.json 2> gpurun_out/${TAG}_gemm_ab.err || exit 3
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python3 -u bench.py ${BENCHARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 4
fi
echo done
