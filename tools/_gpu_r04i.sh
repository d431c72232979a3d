# Round-4: cfg5 training-step kernel profile (DAP weight-gradient reduce after the batched-load fix)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04i
mkdir -p $R
timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $R/prof_train -o run -- python3 tools/train_probe.py 3 3 > $R/train.log 2>&1 || { tail $R/train.log; exit 2; }
f=$(find $R/prof_train -name '*kernel_trace.csv' | head -1); python3 tools/train_profile_summary.py $f 3 > $R/train_summary.json && python3 -c "
import json;d=json.load(open('$R/train_summary.json'));print(json.dumps(d)[:2500])"
find $R -name '*kernel_trace.csv' -size +20M -delete
