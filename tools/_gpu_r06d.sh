# Round 6: OTF row-sweep lookup (tools/_ab/librmd_sweep.so, -DRMD_OTF_SWEEP=1): OTF GPU tests on the
# variant, then per-lookup time A/B against the product at cfg2 and the 4K map (checksums must match)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06d
mkdir -p $R
RMD_LIBRARY=$PWD/tools/_ab/librmd_sweep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/otf_tests.log 2>&1 || { tail -40 $R/otf_tests.log; exit 2; }
tail -2 $R/otf_tests.log
for shape in 8,55,128 2,270,480; do
  for round in 1 2; do
    for v in product sweep; do
      L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; [ $v = sweep ] && L=$PWD/tools/_ab/librmd_sweep.so
      OTF_SHAPE=$shape RMD_LIBRARY=$L timeout -k 10 180 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/t_${v}_${shape}_$round.json 2> $R/t.err || { tail $R/t.err; exit 3; }
      echo "$v $shape $(cat $R/t_${v}_${shape}_$round.json)"
    done
  done
done
echo done
