# fp32-mode OTF lookup: split-bf16 (product) vs exact f32 MFMA (fp32-exact): parity + kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/otfx3
mkdir -p $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_otf.py > $R/tests.log 2>&1 || exit 3
for V in x3 exact; do

  P=fp32; [ $V = exact ] && P=fp32-exact; timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/$V -o run -- python3 tools/otf_probe.py 10 $P > $R/$V.log 2>&1 || exit 4
  python3 tools/trace_summary.py $(find $R/$V -name '*kernel_trace.csv') otf_ > $R/$V.txt
  find $R/$V -name '*kernel_trace.csv' -delete
done
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/bf16 -o run -- python3 tools/otf_probe.py 10 bf16 > $R/bf16.log 2>&1 || exit 5
python3 tools/trace_summary.py $(find $R/bf16 -name '*kernel_trace.csv') otf_ > $R/bf16.txt
find $R/bf16 -name '*kernel_trace.csv' -delete
echo done
