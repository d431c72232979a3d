# L2 behaviour of the cfg2 GEMMs: TCC hit/miss and memory-side requests (one rocprofv3 --pmc pass
# each) for the x3 kernel (product, and RMD_ABLATE=1 = stores dropped) and the w8 kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/l2
mkdir -p $R
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/x3 -o run -- python3 tools/x3_one.py fp32 > $R/x3.log 2>&1 && \
RMD_ABLATE=1 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/x3ns -o run -- python3 tools/x3_one.py fp32 > $R/x3ns.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/w8 -o run -- python3 tools/x3_one.py bf16 > $R/w8.log 2>&1 || exit 5
for p in x3 x3ns w8; do f=$(find $R/$p -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernel.py $f corr_pyramid > $R/$p.json; rm -f $f; done
echo done
