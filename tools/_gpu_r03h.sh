# cfg5 b6 training step (tools/train_probe.py: 3 warm-up, idle gap, 3 timed steps) under rocprofv3
# --kernel-trace; only the summary is kept (the trace is deleted on the box: > 64 MiB)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r03h
mkdir -p $R
timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/r03h_prof -o run -- python3 tools/train_probe.py 3 3 > $R/probe.log 2>&1 || { tail $R/probe.log; exit 3; }
python3 tools/train_profile_summary.py /tmp/r03h_prof/run_kernel_trace.csv 3 > $R/summary.json || exit 4
cat $R/probe.log | tail -2
cat $R/summary.json
