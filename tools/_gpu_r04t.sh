# Round-4: OTF lookup at the 4K map (b2, 270x480) and cfg2: product vs workgroup / block variants
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04t
mkdir -p $R
for shape in 2,270,480 8,55,128; do
  for v in product n512b q16x4n512b product; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    OTF_SHAPE=$shape RMD_LIBRARY=$L timeout -k 10 180 python3 -u tools/otf_time.py 5 bf16 > $R/t.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    python3 -c "import json;d=json.load(open('$R/t.json'));print('$shape', '$v', round(d['bf16']['median_us'],1), d['bf16']['checksum'])"
  done
done
