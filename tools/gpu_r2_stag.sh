#!/bin/bash
# Staggered vs lockstep chain issue (--no-stagger) after the apply-geometry
# change: rank plans P=8/4/2 (twice) and the 1-GPU 16384^2 solve.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/stag
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for rep in 1 2; do
  for P in 8 4 2; do
    for s in stagger lockstep; do
      f=--stagger; [ $s = lockstep ] && f=--no-stagger
      timeout -k 10 300 python -u bench.py --simulate-P $P --n 16384 --sim-sweeps 2 $f \
        --json-out $O/p${P}_${s}_$rep.json > $O/p${P}_${s}_$rep.log 2>&1 || { tail -20 $O/p${P}_${s}_$rep.log; exit 1; }
      echo "P=$P $s rep $rep: $(python3 -c "import json; print(json.load(open('$O/p${P}_${s}_$rep.json'))['value'])")"
    done
  done
done
for s in stagger lockstep; do
  f=--stagger; [ $s = lockstep ] && f=--no-stagger
  timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 $f --json-out $O/one_$s.json \
    > $O/one_$s.log 2>&1 || { tail -20 $O/one_$s.log; exit 1; }
  echo "1-GPU $s: $(python3 -c "import json; d=json.load(open('$O/one_$s.json')); print(d['ms_per_step'])")"
done
