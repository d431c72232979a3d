# Round 6: two half-batch streams vs the sequential step (tools/overlap_ab.py)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06k
mkdir -p $R
timeout -k 10 300 python3 -u tools/overlap_ab.py 30 > $R/overlap.json 2> $R/overlap.err || { tail $R/overlap.err; exit 2; }
cat $R/overlap.json
