#!/bin/bash
# Apply workgroup target (SVDJ_APPLY_WG_TARGET) after the element-wise Q fill:
# rank plans P=8/4/2 and the 1-GPU 16384^2 solve.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/awg2
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for T in ${TS:-128 256 512}; do
  for P in 8 4 2; do
    SVDJ_APPLY_WG_TARGET=$T timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 \
      --sim-sweeps 2 --json-out $O/p${P}_t$T.json > $O/p${P}_t$T.log 2>&1 || { tail -20 $O/p${P}_t$T.log; exit 1; }
    echo "target=$T P=$P: $(python3 -c "import json; print(json.load(open('$O/p${P}_t$T.json'))['value'])")"
  done
done
for T in ${T1:-512 2048}; do
  SVDJ_APPLY_WG_TARGET=$T timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 \
    --json-out $O/one_t$T.json > $O/one_t$T.log 2>&1 || { tail -20 $O/one_t$T.log; exit 1; }
  echo "target=$T 1-GPU: $(python3 -c "import json; d=json.load(open('$O/one_t$T.json')); print(d['ms_per_step'], d['sweeps'])")"
done
