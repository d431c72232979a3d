# Round-4: split-bf16 OTF lookup at the 4K map: 16x2 (product) vs 16x4 query blocks, 512 threads
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04v
mkdir -p $R
for v in product x3q16x4 product x3q16x4; do
  if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
  OTF_SHAPE=2,270,480 RMD_LIBRARY=$L timeout -k 10 180 python3 -u tools/otf_time.py 5 fp32 > $R/t.json 2> $R/t.err || { tail $R/t.err; exit 3; }
  python3 -c "import json;d=json.load(open('$R/t.json'));print('$v', round(d['fp32']['median_us'],1), d['fp32']['checksum'])"
done
