# Round-4 final tree: raft_fs on-the-fly vs volume forward / training at cfg2 b8 and the 4K map (bench_otf)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ah
mkdir -p $R
timeout -k 10 600 python3 -u tools/bench_otf.py --reps 5 > $R/otf_vs_volume.json 2> $R/otf_vs_volume.err || { tail -20 $R/otf_vs_volume.err; exit 2; }
cat $R/otf_vs_volume.json
