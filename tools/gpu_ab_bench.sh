# Interleaved A/B of the headline solve against a base kernel library (dev aid):
# REPS x (new, base) runs of bench.py --steps 3, one JSON summary line each.
# Usage: bash tools/gpu_ab_bench.sh TAG [REPS] [BASE_SO]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}; REPS=${2:-3}; BASE=${3:-tools/ab/libsvdj_hip_base.so}
O=$R/gpurun_out/abb_$TAG
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for r in $(seq 1 $REPS); do
  for v in new base; do
    if [ $v = base ]; then export SVDJ_HIP_LIB=$R/$BASE; else unset SVDJ_HIP_LIB; fi
    timeout -k 10 300 python3 -u $R/bench.py --n ${N:-16384} --steps 3 --warmup 1 --no-verify \
      > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
    tail -1 $O/bench_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $r, d['ms_per_step'], d['sweeps'])"
  done
done
