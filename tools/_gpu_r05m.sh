# Round 5: OTF forward — bf16 tasks as pairs of adjacent target segments (product) vs single segments (nopair);
# cfg2 and the 4K map; OTF parity tests first
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05m
mkdir -p $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for rep in 1 2; do
  for v in product nopair; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "otf cfg2 $v $rep $(cat $R/t_${v}_$rep.json)"
    OTF_SHAPE=2,270,480 RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/otf_time.py 5 bf16 > $R/k_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 4; }
    echo "otf 4k $v $rep $(cat $R/k_${v}_$rep.json)"
  done
done
