set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/graph_step_ab.py 5 > gpurun_out/graph_ab.json 2> gpurun_out/graph_ab.err
