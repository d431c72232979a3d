# Lookup position effect: which part of the bench step's rising lookup times follows the coords
# (reverse order, coords[11] throughout, a tiny per-position shift) and which the position after the GEMM
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06p}
mkdir -p $R
M=bench,rev,shift,const11,samecoord,nogemm
for round in 1 2; do
  LOOKUP_CONTEXT_MODES=$M timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
    -d $R/ctx_$round -o run -- python3 tools/lookup_context.py 10 > $R/ctx_$round.out 2>&1 || { tail $R/ctx_$round.out; exit 2; }
  f=$(ls $R/ctx_$round/*kernel_trace.csv $R/ctx_$round/*/*kernel_trace.csv 2>/dev/null | head -1)
  LOOKUP_CONTEXT_MODES=$M python3 tools/lookup_context.py --summary $f | tee -a $R/summary.txt
done
echo done
