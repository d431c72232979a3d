# A/B of OTF lookup variants selected by RMD_OTF_ABLATE: kernel durations from rocprofv3 per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 3}; do
  LDSB=""; case $v in *_*) LDSB=${v#*_};; esac
  RMD_OTF_ABLATE=${v%%_*} RMD_OTF_LDS=${LDSB:-} timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/otf_ab/v$v -o run -- python3 tools/otf_probe.py 10 > gpurun_out/otf_ab_$v.log 2>&1 || exit $?
done
