# Round 6: 8-rank rehearsal of bench.py's N-GPU path on one GPU (gloo; the ranks share the card, so only
# the launcher, job-time MAX, live PMC on rank 0 and the JSON line are exercised, not scaling)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r06l
mkdir -p $R
timeout -k 10 900 python3 -u bench.py --gpus 8 --backend gloo --one-device --steps 5 --warmup 2 --fp32-steps 3 \
  --model-level off --train off --hybrid off --dicl off --highres off --no-cpu-baseline > $R/bench8.json 2> $R/bench8.err || { tail -30 $R/bench8.err; exit 2; }
python3 -c "
import json;d=json.loads([l for l in open('$R/bench8.json').read().splitlines() if l.startswith('{')][-1])
print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d['roofline']['traffic_source'][:70], d['fp32_mode']['value'])"
