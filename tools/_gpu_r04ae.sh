# Round-4: OTF lookup on the 4K map (b2, 270x480): wide-map block variants (16 x WQY at WNT threads)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/r04ae
mkdir -p $R
for rep in 1 2; do
  for v in product w8n1024 w6n768 w4n768; do
    if [ $v = product ]; then L=$PWD/raft-meets-dicl_amd/rmd/librmd.so; else L=$PWD/tools/_ab/librmd_$v.so; fi
    OTF_SHAPE=2,270,480 RMD_LIBRARY=$L timeout -k 10 180 python3 -u tools/otf_time.py 5 bf16 > $R/t_${v}_$rep.json 2> $R/t.err || { tail $R/t.err; exit 3; }
    python3 -c "import json;d=json.load(open('$R/t_${v}_$rep.json'));print('$v', $rep, round(d['bf16']['median_us'],1), d['bf16']['checksum'])"
  done
done
