# lookup ablations (diag build): product / no output traffic / no pyramid loads, with moving and with
# repeated coordinates
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so
export RMD_AB="${AB:-V=3,V=2,RMD_ABLATE=3}"
timeout -k 10 300 python3 -u tools/lookup_ab.py 20 bf16 > gpurun_out/lkabl_move.json 2> gpurun_out/lkabl.err || exit 3
LOOKUP_AB_SAME=1 timeout -k 10 300 python3 -u tools/lookup_ab.py 20 bf16 > gpurun_out/lkabl_same.json 2>> gpurun_out/lkabl.err || exit 4
echo done
