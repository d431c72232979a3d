# Component kernels of the non-headline §8 rows (tools/bench_components.py): event timings and live HBM
# traffic per dispatch from separate FETCH_SIZE / WRITE_SIZE counter passes
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06s}
mkdir -p $R
timeout -k 10 400 python3 -u tools/bench_components.py 20 > $R/components.json 2> $R/components.err || { tail -20 $R/components.err; exit 2; }
echo components ok
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pf -o run -- python3 tools/bench_components.py 3 > $R/pf.out 2>&1 || { tail $R/pf.out; exit 3; }
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pw -o run -- python3 tools/bench_components.py 3 > $R/pw.out 2>&1 || { tail $R/pw.out; exit 4; }
python3 tools/pmc_traffic_by_kernel.py $(ls $R/pf/*counter_collection.csv $R/pf/*/*counter_collection.csv 2>/dev/null | head -1) \
    $(ls $R/pw/*counter_collection.csv $R/pw/*/*counter_collection.csv 2>/dev/null | head -1) | tee $R/traffic.jsonl
echo done
