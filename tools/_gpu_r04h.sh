# Round-4: cache-policy A/B in the bench context (GEMM + 12 lookups per step): VARIANTS = tools/_ab builds
# sc0 = 1, nt = 2 (product), sc1 = 16; kernel-trace mean over positions per build
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04h
mkdir -p $R
export LOOKUP_CONTEXT_MODES=bench
for v in $VARIANTS; do
  lib=$PWD/raft-meets-dicl_amd/rmd/librmd.so; [ $v != product ] && lib=$PWD/tools/_ab/librmd_$v.so
  RMD_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/ctx_$v -o run -- python3 tools/lookup_context.py 10 > $R/ctx_$v.log 2>&1 || { tail $R/ctx_$v.log; exit 2; }
  f=$(find $R/ctx_$v -name '*kernel_trace.csv' | head -1)
  echo "$v $(python3 tools/lookup_context.py --summary $f)" | tee -a $R/ctx.jsonl
  rm -rf $R/ctx_$v
done
