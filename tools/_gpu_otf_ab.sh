# OTF lookup A/B at cfg2: tools/_gpu_otf_ab.sh OUTDIR "variant ..." (variant = product or tools/_ab/librmd_<v>.so),
# two interleaved passes; GPU OTF tests of the product build first
set -o pipefail
export TMPDIR=/tmp
R=$1
mkdir -p $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_otf.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 2; }
tail -1 $R/tests.log
for rep in 1 2; do
  for v in $2; do
    O=$R/t_${v}_${rep}.json
    if [ $v = product ]; then
      timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 fp32 > $O 2> $R/t_${v}.err || { tail $R/t_${v}.err; exit 3; }
    else
      RMD_LIBRARY=$PWD/tools/_ab/librmd_$v.so timeout -k 10 120 python3 -u tools/otf_time.py 10 bf16 fp32 > $O 2> $R/t_${v}.err || { tail $R/t_${v}.err; exit 3; }
    fi
    python3 -c "import json;d=json.load(open('$O'));print('$v', $rep, round(d['bf16']['median_us'],1), round(d['fp32']['median_us'],1), d['bf16']['checksum'], d['fp32']['checksum'])"
  done
done
