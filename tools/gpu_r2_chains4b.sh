#!/bin/bash
# Four chains: stagger modes (SVDJ_STAGGER_N 0 cascade, 1 pairs, 2 none).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/chains4b
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for sm in 1 2; do
  for cfg in ${CFGS:-8:64 4:64}; do
    set -- ${cfg//:/ }
    SVDJ_STAGGER_N=$sm timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --block $2 --chains 4 --json-out $O/s${sm}_p$1_w$2.json > $O/s${sm}_p$1_w$2.log 2>&1 || { tail -20 $O/s${sm}_p$1_w$2.log; exit 1; }
    echo "stagger=$sm P=$1 W=$2 chains=4: $(python3 -c "import json; print(json.load(open('$O/s${sm}_p$1_w$2.json'))['value'])")"
  done
done
