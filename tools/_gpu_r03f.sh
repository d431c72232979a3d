# OTF 4K A/B (product vs the round-2 block shape) and the cfg2 whole-volume cross-kernel test
set -o pipefail
R=gpurun_out/r03f
mkdir -p $R
timeout -k 10 300 python3 -u tools/bench_otf.py --reps 5 > $R/otf_product.json 2> $R/otf.err || { tail $R/otf.err; exit 4; }
RMD_LIBRARY=$PWD/tools/_bin/librmd_otf_r2shape.so timeout -k 10 300 python3 -u tools/bench_otf.py --reps 5 > $R/otf_r2shape.json 2>> $R/otf.err || exit 5
cat $R/otf_product.json; echo; cat $R/otf_r2shape.json; echo
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k whole_volume --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 6; }
tail -2 $R/tests.log
