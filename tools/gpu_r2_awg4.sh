#!/bin/bash
# Finer apply workgroup targets: 2-GPU plan (32 pairs/step), 1-GPU 16384^2
# (64 pairs/step) and 4096^2 (W=32).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/awg4
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for T in 256 1024; do
  SVDJ_APPLY_WG_TARGET=$T timeout -k 10 300 python -u bench.py --simulate-P 2 --simulate-rank 0 --n 16384 \
    --sim-sweeps 2 --json-out $O/p2_t$T.json > $O/p2_t$T.log 2>&1 || { tail -20 $O/p2_t$T.log; exit 1; }
  echo "target=$T P=2: $(python3 -c "import json; print(json.load(open('$O/p2_t$T.json'))['value'])")"
done
for T in 1024 4096; do
  SVDJ_APPLY_WG_TARGET=$T timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 \
    --json-out $O/one_t$T.json > $O/one_t$T.log 2>&1 || { tail -20 $O/one_t$T.log; exit 1; }
  echo "target=$T 1-GPU 16384: $(python3 -c "import json; d=json.load(open('$O/one_t$T.json')); print(d['ms_per_step'])")"
  SVDJ_APPLY_WG_TARGET=$T timeout -k 10 300 python -u bench.py --n 4096 --steps 3 --warmup 1 \
    --json-out $O/f4096_t$T.json > $O/f4096_t$T.log 2>&1 || { tail -20 $O/f4096_t$T.log; exit 1; }
  echo "target=$T 4096: $(python3 -c "import json; d=json.load(open('$O/f4096_t$T.json')); print(d['ms_per_step'])")"
done
