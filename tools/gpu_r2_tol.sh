#!/bin/bash
# Stop-threshold experiment: default 4 sqrt(m) eps vs sqrt(m) eps (LAPACK
# xGESVJ) and 2 sqrt(m) eps, fp32, 4096^2 and 16384^2: time, sweeps, accuracy.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tol
export SVDJ_NO_AUTOBUILD=1
for N in 4096 16384; do
  for f in 4 2 1; do
    TOL=$(python3 -c "import math; print($f * math.sqrt($N) * 2**-23)")
    timeout -k 10 300 python -u bench.py --n $N --steps 1 --warmup 1 --tol $TOL \
      --json-out gpurun_out/tol/n${N}_f$f.json > gpurun_out/tol/n${N}_f$f.log 2>&1 || { tail -20 gpurun_out/tol/n${N}_f$f.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/tol/n${N}_f$f.json')); print($N, $f, d['ms_per_step'], d['sweeps'], d['accuracy'])"
  done
done
