# Round-4: lookup time by position in the bench step under four contexts (tools/lookup_context.py)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04g
mkdir -p $R
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/ctx -o run -- python3 tools/lookup_context.py 10 > $R/ctx.log 2>&1 || { tail $R/ctx.log; exit 2; }
f=$(find $R/ctx -name '*kernel_trace.csv' | head -1)
python3 tools/lookup_context.py --summary $f | tee $R/ctx.json
find $R -name '*kernel_trace.csv' -size +20M -delete
