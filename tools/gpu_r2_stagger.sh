#!/bin/bash
# Symmetric vs one-sided chain stagger (SVDJ_STAGGER_SYM) x Gram chunk target
# on the 8-GPU rank plans and the one-GPU headline.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/stagger
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for sym in 1 0; do
  for cfg in ${CFGS:-8:32:512 8:32:1024 8:64:512 4:64:512}; do
    set -- ${cfg//:/ }
    SVDJ_STAGGER_SYM=$sym SVDJ_GRAM_WG_TARGET=$3 timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 \
      --n 16384 --sim-sweeps 2 --block $2 --json-out $O/s${sym}_$1_$2_$3.json > $O/s${sym}_$1_$2_$3.log 2>&1 \
      || { tail -20 $O/s${sym}_$1_$2_$3.log; exit 1; }
    echo "sym=$sym P=$1 W=$2 gram=$3: $(python3 -c "import json; print(json.load(open('$O/s${sym}_$1_$2_$3.json'))['value'])")"
  done
  SVDJ_STAGGER_SYM=$sym timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --no-verify \
    --json-out $O/one_s$sym.json > $O/one_s$sym.log 2>&1 || { tail -20 $O/one_s$sym.log; exit 1; }
  echo "sym=$sym 1-GPU 16384: $(python3 -c "import json; d=json.load(open('$O/one_s$sym.json')); print(d['ms_per_step'], d['sweeps'])")"
done
