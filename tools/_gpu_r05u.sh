# Round 5: 2-rank rehearsal of the bench launcher on one GPU (gloo, --one-device: live PMC traffic and the
# MFMA-busy pass from rank 0, rank 0's cpu_baseline); OTF lookup counters at cfg2 bf16 (three passes)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r05u
mkdir -p $R
timeout -k 10 500 python3 -u bench.py --gpus 2 --backend gloo --one-device --steps 10 --warmup 3 --model-level off --dicl off --hybrid off --train off --highres off --fp32-mode off --cpu-budget-s 3 > $R/rehearse2.json 2> $R/rehearse2.err || { tail -20 $R/rehearse2.err; exit 3; }
python3 -c "import json;d=json.loads(open('$R/rehearse2.json').read().splitlines()[-1]);print('rehearse2', d['value'],d['n_gpus'],d['roofline']['traffic_source'][:60],d['roofline']['traffic'],d['roofline_gemm'].get('mfma_busy'),d['cpu_baseline']['value'],d['cpu_baseline'].get('note'))"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P3="TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/otf_p$i -o run -- python3 tools/otf_time.py 2 bf16 > /dev/null 2> $R/otf_p$i.err || { tail -5 $R/otf_p$i.err; exit 4; }
  python3 tools/pmc_kernel.py $R/otf_p$i/run_counter_collection.csv otf_lookup > $R/otf_p$i.json
  cat $R/otf_p$i.json | head -30
done
find $R -name '*.csv' -size +4M -delete
