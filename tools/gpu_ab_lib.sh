# A/B of two builds of the kernel library on one GPU (development aid).
# Usage: bash tools/gpu_ab_lib.sh BASE_SO TAG [bench args]
#   BASE_SO: an alternative libsvdj_hip.so (e.g. tools/ab/libsvdj_hip_base.so built
#   from HEAD's sources); the in-tree build is "new".  Per build: tools/step_probe.py
#   (copy bandwidth, per-step time) and one 16384^2 bench solve; logs under
#   gpurun_out/ab_TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
BASE=$1; TAG=$2; shift 2; EXTRA="$@"
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for v in new base; do
  if [ $v = base ]; then export SVDJ_HIP_LIB=$R/$BASE; else unset SVDJ_HIP_LIB; fi
  timeout -k 10 240 python -u $R/tools/step_probe.py > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
  cat $O/probe_$v.log
  timeout -k 10 300 python -u $R/bench.py --n 16384 --steps 1 --warmup 0 --progress $EXTRA > $O/bench_$v.log 2>&1 \
    || { tail -20 $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | cut -c1-420
done
