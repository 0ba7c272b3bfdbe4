#!/bin/bash
# Inner EVD sweeps per pair (max_inner_sweeps) vs outer sweeps and time.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/inner
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for n in ${NS:-4096 16384}; do
  for k in ${KS:-1 2 3}; do
    timeout -k 10 300 python -u bench.py --n $n --steps 1 --warmup 1 --inner $k --json-out $O/n${n}_i$k.json > $O/n${n}_i$k.log 2>&1 || { tail -20 $O/n${n}_i$k.log; exit 1; }
    echo "n=$n inner=$k: $(python3 -c "import json; d=json.load(open('$O/n${n}_i$k.json')); print(d['ms_per_step'], d['sweeps'], d['accuracy'])")"
  done
done
