# VERDICT r05 hygiene: rebuild librmd.so from a clean csrc/ ON the GPU box, compare it with the
# library shipped in the tree (sha256 + source fingerprint), then run the GPU suite, smoke and the
# default bench line against the box-built library
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/${RUN:-r06n}
mkdir -p $R
LIB=raft-meets-dicl_amd/rmd/librmd.so
sha256sum $LIB | tee $R/shipped.sha256
make -C raft-meets-dicl_amd/csrc clean > $R/build.log 2>&1 && \
  timeout -k 10 600 make -C raft-meets-dicl_amd/csrc -j16 >> $R/build.log 2>&1 || { tail -20 $R/build.log; exit 2; }
sha256sum $LIB | tee $R/boxbuilt.sha256
python3 -c "
import sys; sys.path.insert(0, 'raft-meets-dicl_amd')
from rmd import _lib; i = _lib.build_info(); print('build_info', i); assert i['sources_match']" | tee $R/build_info.txt || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 4; }
tail -2 $R/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail $R/smoke.log; exit 5; }
tail -4 $R/smoke.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 6; }
python3 -c "
import json;d=json.loads(open('$R/bench.json').read().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline_gemm']['avg_launch_ms'])
f=d['fp32_mode']; print('fp32', f['value'], f['roofline_gemm']['avg_launch_ms'], f['roofline_gemm'].get('mfma_busy'))
print('library', d['library']); print('dicl', d['dicl_matching'].get('volume_gbps'))"
echo done
