# Round 5: G build variants — non-temporal G stores (nt), 1-row tiles (rb1), 2-chunk tiles (cb2nt)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${1:-r05ze}
mkdir -p $R
for v in product scb2 srb1 sg2 scb8; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  RMD_LIBRARY=$L timeout -k 10 120 python3 -u tools/bench_grad_build.py 20 > $R/gb_$v.jsonl 2> $R/gb.err || { tail -5 $R/gb.err; exit 3; }
  echo "== $v"; cat $R/gb_$v.jsonl
done
