# Round 5: OTF lookup with a software-pipelined task loop (pf: next task's fragments in flight during this
# task's MFMAs, 118 VGPRs, 4 waves/SIMD) vs the product; OTF tests on the variant first
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05v
mkdir -p $R
RMD_LIBRARY=$PWD/tools/_ab/librmd_pf.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for rep in 1 2 3; do
  for v in product pf; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "otf cfg2 $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
OTF_SHAPE=2,270,480 RMD_LIBRARY=$PWD/tools/_ab/librmd_pf.so timeout -k 10 120 python3 -u tools/otf_time.py 5 bf16 > $R/k_pf.json 2> $R/t.err || { tail $R/t.err; exit 4; }
OTF_SHAPE=2,270,480 timeout -k 10 120 python3 -u tools/otf_time.py 5 bf16 > $R/k_product.json 2> $R/t.err || { tail $R/t.err; exit 4; }
echo "4k pf $(cat $R/k_pf.json)"; echo "4k product $(cat $R/k_product.json)"
