#!/bin/bash
# Block width vs GPU count with the bipartite cross-step EVD (default since
# round 2): simulated rank plans of 16384^2 (P = 2, 4, 8) and 65536^2 (P = 8),
# one-GPU 8192^2 / 12288^2 solves, W = 32 vs 64.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/simgrid2
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for cfg in ${CFGS:-"16384 2" "16384 4" "16384 8"}; do
  set -- $cfg
  for W in 32 64; do
    timeout -k 10 300 python -u bench.py --simulate-P $2 --simulate-rank 0 --n $1 --sim-sweeps 2 --block $W \
      --json-out $O/sim_n$1_p$2_w$W.json > $O/sim_n$1_p$2_w$W.log 2>&1 || { tail -20 $O/sim_n$1_p$2_w$W.log; exit 1; }
    echo "n=$1 P=$2 W=$W: $(python3 -c "import json; print(json.load(open('$O/sim_n$1_p$2_w$W.json'))['value'])") ms/sweep"
  done
done
for n in ${ONE:-4096 8192 12288}; do
  for W in 32 64; do
    timeout -k 10 300 python -u bench.py --n $n --steps 1 --warmup 1 --block $W --json-out $O/one_${n}_w$W.json \
      > $O/one_${n}_w$W.log 2>&1 || { tail -20 $O/one_${n}_w$W.log; exit 1; }
    echo "1-GPU n=$n W=$W: $(python3 -c "import json; d=json.load(open('$O/one_${n}_w$W.json')); print(d['ms_per_step'], 'ms', d['sweeps'])")"
  done
done
