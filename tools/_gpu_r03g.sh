# lookup buffer-load fast path: GPU corr tests on the product library, then a same-box A/B vs the pointer path
set -o pipefail
R=gpurun_out/r03g
mkdir -p $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_corr.py tests/test_gpu_graph.py tests/test_gpu_e2e.py tests/test_library.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 3; }
tail -2 $R/tests.log
run() { RMD_LIBRARY=$1 timeout -k 10 300 python3 -u tools/lookup_time.py 20 >> $R/ab.jsonl 2>> $R/err.log; }
rm -f $R/ab.jsonl
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 4
run $PWD/tools/_bin/librmd_lookup_ptr.so || exit 5
run $PWD/raft-meets-dicl_amd/rmd/librmd.so || exit 6
run $PWD/tools/_bin/librmd_lookup_ptr.so || exit 7
cat $R/ab.jsonl
