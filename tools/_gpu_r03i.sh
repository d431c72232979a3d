# OTF bf16 task prefetch A/B (16x1 blocks, 2 WG/CU) + cfg5 training-step profile
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r03i
mkdir -p $R
run() { RMD_LIBRARY=$1 timeout -k 10 300 python3 -u tools/otf_time.py 10 bf16 >> $R/otf_ab.jsonl 2>> $R/err.log; }
rm -f $R/otf_ab.jsonl
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 3
run $PWD/tools/_bin/librmd_otf_pf_o2.so || exit 4
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 5
run $PWD/tools/_bin/librmd_otf_pf_o2.so || exit 6
cat $R/otf_ab.jsonl
bash tools/_gpu_r03h.sh
