# OTF lookup: target-fragment prefetch A/B (diag build), kernel durations by rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so
R=gpurun_out/otfpf
mkdir -p $R
for PF in 0 1; do
  for A in 0 3; do
    RMD_OTF_PF=$PF RMD_OTF_ABLATE=$A timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/p${PF}a$A -o run -- python3 tools/otf_probe.py 10 ${PREC:-bf16} > $R/p${PF}a$A.log 2>&1 || exit 3
    echo "PF=$PF ABLATE=$A $(python3 tools/trace_summary.py $(find $R/p${PF}a$A -name '*kernel_trace.csv') otf_lookup)" >> $R/summary.txt
    find $R/p${PF}a$A -name '*kernel_trace.csv' -delete
  done
done
echo done
