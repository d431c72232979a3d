# Round 6: debug the S24 epilogue (permlane semantics probe + per-level diff)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06c
mkdir -p $R
timeout -k 10 60 tools/_ab/perm_probe > $R/perm.txt 2>&1 || { cat $R/perm.txt; exit 2; }
cat $R/perm.txt
timeout -k 10 120 python3 -u tools/s24_debug.py 2 32 24 40 > $R/s24.txt 2>&1 || { tail -30 $R/s24.txt; exit 3; }
cat $R/s24.txt
