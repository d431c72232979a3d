# Round-4: OTF backward G build by owner threads (product) vs per-(query, column) sums (bwdprev): OTF GPU
# tests, bitwise comparison of the cfg2 gradients of both builds, bench_otf training times
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04aj
mkdir -p $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_otf.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for p in bf16 fp32; do
  timeout -k 10 120 python3 tools/otf_bwd_dump.py $R/new_$p.npz $p && RMD_LIBRARY=$PWD/tools/_ab/librmd_bwdprev.so timeout -k 10 120 python3 tools/otf_bwd_dump.py $R/old_$p.npz $p || exit 3
  python3 -c "
import numpy as np; a=np.load('$R/new_$p.npz'); b=np.load('$R/old_$p.npz')
print('$p bitwise equal:', all(np.array_equal(a[k], b[k]) for k in ('g1','g2')))"
done
for v in product bwdprev product bwdprev; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -k 10 300 python3 -u tools/bench_otf.py --reps 3 --skip-4k > $R/b_$v.json 2> $R/b_$v.err || { tail $R/b_$v.err; exit 4; }
  python3 -c "
import json;d=json.load(open('$R/b_$v.json'));print('$v', {k: round(v['otf_backward_ms'],2) for k, v in d.items() if 'otf_backward_ms' in v})"
done
rm -f $R/*.npz
