#!/bin/bash
# Remaining block-width points with the bipartite EVD: fp64 one-GPU solves,
# the 8-GPU rank plans of 8192^2 and 65536^2 fp32.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/simgrid3
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for W in 32 64; do
  for n in 5000 8192; do
    timeout -k 10 300 python -u bench.py --n $n --dtype fp64 --steps 1 --warmup 1 --block $W --json-out $O/fp64_${n}_w$W.json \
      > $O/fp64_${n}_w$W.log 2>&1 || { tail -20 $O/fp64_${n}_w$W.log; exit 1; }
    echo "1-GPU fp64 n=$n W=$W: $(python3 -c "import json; d=json.load(open('$O/fp64_${n}_w$W.json')); print(d['ms_per_step'], 'ms', d['sweeps'])")"
  done
done
for cfg in "8192 8" "65536 8"; do
  set -- $cfg
  for W in 32 64; do
    timeout -k 10 300 python -u bench.py --simulate-P $2 --simulate-rank 0 --n $1 --sim-sweeps 1 --block $W \
      --json-out $O/sim_n$1_p$2_w$W.json > $O/sim_n$1_p$2_w$W.log 2>&1 || { tail -20 $O/sim_n$1_p$2_w$W.log; exit 1; }
    echo "n=$1 P=$2 W=$W: $(python3 -c "import json; print(json.load(open('$O/sim_n$1_p$2_w$W.json'))['value'])") ms/sweep"
  done
done
