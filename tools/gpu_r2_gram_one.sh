#!/bin/bash
# Gram split-K chunk count on one-GPU solves: SVDJ_GRAM_WG_TARGET sweep.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/gram_one
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for n in ${NS:-8192 16384}; do
  for T in ${TS:-512 2048 4096}; do
    SVDJ_GRAM_WG_TARGET=$T timeout -k 10 300 python -u bench.py --n $n --steps 1 --warmup 1 --no-verify \
      --json-out $O/n${n}_t$T.json > $O/n${n}_t$T.log 2>&1 || { tail -20 $O/n${n}_t$T.log; exit 1; }
    echo "n=$n target=$T: $(python3 -c "import json; d=json.load(open('$O/n${n}_t$T.json')); print(d['ms_per_step'], d['sweeps'])")"
  done
done
