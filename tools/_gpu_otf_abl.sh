# OTF lookup ablations (diag build): kernel durations by rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so
R=gpurun_out/otfabl
mkdir -p $R
for A in 0 1 2 3; do
  RMD_OTF_ABLATE=$A timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/a$A -o run -- python3 tools/otf_probe.py 10 bf16 > $R/a$A.log 2>&1 || exit 3
  python3 tools/trace_summary.py $(find $R/a$A -name '*kernel_trace.csv') otf_lookup > $R/a$A.txt
  find $R/a$A -name '*kernel_trace.csv' -delete
done
echo done
