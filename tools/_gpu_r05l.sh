# Round 5: OTF forward — per-segment task skips (product) vs none (noskip), query fragments in registers
# (qreg, qreg4y = 16x4 blocks), 16x4 blocks at 512 threads (w4y); OTF parity tests first
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05l
mkdir -p $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_otf.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 2; }
tail -2 $R/tests.log
for rep in 1 2; do
  for v in product noskip qreg qreg4y w4y; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    echo "otf $v $rep $(cat $R/t_${v}_$rep.json)"
  done
done
