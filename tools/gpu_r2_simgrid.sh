#!/bin/bash
# Simulated per-rank sweep time of the 16384^2 fp32 job at P = 2, 4, 8 for
# block widths 32 and 64 (rank 0's real plan on one GPU, exchanges as device
# copies): which W the per-GPU column count should pick.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/simgrid
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for P in ${PS:-2 4 8}; do
  for W in ${WS:-32 64}; do
    timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n ${N:-16384} --sim-sweeps 2 --block $W \
      --json-out $O/sim_p${P}_w$W.json > $O/sim_p${P}_w$W.log 2>&1 || { tail -20 $O/sim_p${P}_w$W.log; exit 1; }
    echo "P=$P W=$W: $(python3 -c "import json; d=json.load(open('$O/sim_p${P}_w$W.json')); print(d['value'], d['unit'])")"
  done
done
