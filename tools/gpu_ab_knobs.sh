# Interleaved A/B of SVDJ_DEBUG settings on the headline solve (dev aid):
# REPS rounds over the variants (bench.py --steps 3, no verify), then one
# verified run per variant for the accuracy block.  One summary line per run.
# Usage: bash tools/gpu_ab_knobs.sh TAG REPS "variant1" "variant2" ...
#        (a variant is an SVDJ_DEBUG value, "-" = unset, optionally followed by
#        "@" and extra bench.py arguments, e.g. "merge=1@--quad on")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; REPS=$2; shift 2
O=$R/gpurun_out/abk_$TAG
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); a=d.get("accuracy") or {}; print(sys.argv[1], d["ms_per_step"], d["sweeps"], a.get("residual_rel"), a.get("orth_u_max_abs"), a.get("orth_v_max_abs"), flush=True)'
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    k=${v%%@*}; x=""; [ "$k" != "$v" ] && x=${v#*@}
    if [ "$k" = "-" ]; then unset SVDJ_DEBUG; else export SVDJ_DEBUG="$k"; fi
    timeout -k 10 300 python3 -u $R/bench.py --n ${N:-16384} --steps ${STEPS:-3} --warmup 1 --no-verify $x \
      > $O/bench_${i}_$r.log 2>&1 || { tail -20 $O/bench_${i}_$r.log; exit 1; }
    tail -1 $O/bench_${i}_$r.log | python3 -c "$summ" "$v/$r"
  done
done
i=0
for v in "$@"; do
  i=$((i+1))
  k=${v%%@*}; x=""; [ "$k" != "$v" ] && x=${v#*@}
  if [ "$k" = "-" ]; then unset SVDJ_DEBUG; else export SVDJ_DEBUG="$k"; fi
  timeout -k 10 400 python3 -u $R/bench.py --n ${N:-16384} --steps 1 --warmup 0 $x \
    > $O/acc_${i}.log 2>&1 || { tail -20 $O/acc_${i}.log; exit 1; }
  tail -1 $O/acc_${i}.log | python3 -c "$summ" "$v/acc"
done
