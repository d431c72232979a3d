# Round-4: OTF product build (wide-map 16x4 dispatch, split-bf16 at 512 threads): GPU OTF tests, timing
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04u
mkdir -p $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_otf.py -x -v --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for shape in 2,270,480 8,55,128; do
  OTF_SHAPE=$shape timeout -k 10 180 python3 -u tools/otf_time.py 10 bf16 fp32 > $R/t_$shape.json 2> $R/t.err || { tail $R/t.err; exit 3; }
  cat $R/t_$shape.json
done
