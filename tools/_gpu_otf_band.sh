set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/otfband
mkdir -p $R
RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag_otf256.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_otf.py > $R/tests256.log 2>&1 || exit 3
for L in librmd_diag librmd_diag_otf256; do
  RMD_LIBRARY=raft-meets-dicl_amd/rmd/$L.so timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/$L -o run -- python3 tools/otf_probe.py 10 bf16 > $R/$L.log 2>&1 || exit 4
  python3 tools/trace_summary.py $(find $R/$L -name '*kernel_trace.csv') otf_lookup > $R/$L.txt
  find $R/$L -name '*kernel_trace.csv' -delete
done
echo done
