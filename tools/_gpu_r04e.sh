# Round-4: lookup A/B (h64 = b64 half-row loads; h64w8 = + 8 waves/SIMD; nold / nost / notr = h64 with
# loads / stores / both sent to kOOB through a runtime global: the valid no-traffic floor), then the
# whole GPU suite on this tree, then a 2-rank gloo rehearsal on one GPU (live PMC + cpu_baseline at N>1)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04e
mkdir -p $R
P=$PWD/raft-meets-dicl_amd/rmd/librmd.so
B=$PWD/tools/_ab
run() { RMD_LIBRARY=$1 timeout -k 10 120 python3 -u tools/lookup_time.py 30 bf16 >> $R/lookup_ab.jsonl 2>> $R/err.log; }
run $P || exit 3
for v in h64 h64w8 nold nost notr; do run $B/librmd_$v.so || exit 4; done
run $P || exit 5
for v in h64w8 h64; do run $B/librmd_$v.so || exit 6; done
cat $R/lookup_ab.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 7; }
tail -3 $R/tests.log
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --one-device --steps 10 --warmup 3 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --cpu-budget-s 3 > $R/rehearse2.json 2> $R/rehearse2.err || { tail -20 $R/rehearse2.err; exit 8; }
python3 -c "import json;d=json.loads(open('$R/rehearse2.json').read().splitlines()[-1]);print(d['value'],d['n_gpus'],d['roofline']['traffic_source'],d['roofline']['traffic'],d['cpu_baseline']['value'],d['cpu_baseline'].get('note'))"
