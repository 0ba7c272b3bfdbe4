#!/bin/bash
# Apply grid sizing: SVDJ_APPLY_WG_TARGET (workgroups the apply aims for per
# launch) on simulated rank plans of the 16384^2 fp32 job.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/apply_wg
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for cfg in ${CFGS:-1:64 2:64 8:32}; do   # P:W
  set -- ${cfg/:/ }
  for T in ${TS:-512 1024 2048 4096}; do
    env ${VAR:-SVDJ_APPLY_WG_TARGET}=$T timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 \
      --sim-sweeps 2 --block $2 --json-out $O/p$1_w$2_t$T.json > $O/p$1_w$2_t$T.log 2>&1 || { tail -20 $O/p$1_w$2_t$T.log; exit 1; }
    echo "P=$1 W=$2 target=$T: $(python3 -c "import json; d=json.load(open('$O/p$1_w$2_t$T.json')); print(d['value'])")"
  done
done
