# Interleaved A/B of rank plans (bench.py --simulate-P, one GPU) over
# SVDJ_DEBUG settings and bench arguments (dev aid).
# Usage: N=16384 P=8 bash tools/gpu_ab_sim.sh TAG REPS "variant1" ...
#        (variant: SVDJ_DEBUG value, "-" = unset, optionally "@" + bench args)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; REPS=$2; shift 2
O=$R/gpurun_out/abs_$TAG
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], d["value"], "ms/sweep quad", d["config"]["quad_steps"], flush=True)'
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    k=${v%%@*}; x=""; [ "$k" != "$v" ] && x=${v#*@}
    if [ "$k" = "-" ]; then unset SVDJ_DEBUG; else export SVDJ_DEBUG="$k"; fi
    timeout -k 10 300 python3 -u $R/bench.py --n ${N:-16384} --simulate-P ${P:-8} --sim-sweeps ${SW:-3} $x \
      > $O/sim_${i}_$r.log 2>&1 || { tail -20 $O/sim_${i}_$r.log; exit 1; }
    tail -1 $O/sim_${i}_$r.log | python3 -c "$summ" "$v/$r"
  done
done
