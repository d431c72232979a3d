# Round-4: x3 GEMM (fp32 mode) on one box: product vs free-running phases (x3pp0), stores dropped (x3abl1,
# wrong results), epilogue + stores without the k-loop (x3abl2, wrong results)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04am
mkdir -p $R
for rep in 1 2; do
  for v in product x3pp0 x3abl1 x3abl2; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/x3_time.py 20 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "$v $rep $(cat $R/t_${v}_$rep.json | head -c 250)"
  done
done
