set -o pipefail
cd $GRAFT_REPO_ROOT
RMD_LOOKUP_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lookup or corr_block or golden" > gpurun_out/split2_tests.log 2>&1 &&
RMD_LOOKUP_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lookup or corr_block or golden" > gpurun_out/split1_tests.log 2>&1 &&
RMD_AB=0,1,1:3,1:2,1:1 timeout -k 10 200 python -u tools/lookup_ab.py 20 > gpurun_out/lookup_ab_split.json 2> gpurun_out/lookup_ab_split.err
