# Round-6 quad rule check (dev aid): the default plans after the rule change
# (one simulated run each), then the full GPU suite and smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rule
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
for c in "16384 2" "16384 4" "16384 8" "8192 2" "12288 4" "8192 4"; do
  set -- $c
  timeout -k 10 300 python3 -u bench.py --n $1 --simulate-P $2 --sim-sweeps 3 > $O/plan_${1}_P$2.log 2>&1 || { tail -20 $O/plan_${1}_P$2.log; exit 1; }
  tail -1 $O/plan_${1}_P$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 P=$2', d['value'], 'ms/sweep quad', d['config']['quad_steps'])"
done
bash tools/gpu_full.sh
