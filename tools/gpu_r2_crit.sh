#!/bin/bash
# Critical-path split (wide kernels / EVD-only / idle) of simulated rank plans
# of 16384^2 fp32 at P = 1, 2, 4, 8 (tools/trace_crit.py).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/crit
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-8:64}; do   # P:W
  set -- ${cfg/:/ }
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$1_w$2 -o run -- python $R/bench.py --simulate-P $1 \
    --simulate-rank 0 --n ${N:-16384} --sim-sweeps 2 --block $2 > $O/p$1_w$2.log 2>&1 || { tail -20 $O/p$1_w$2.log; exit 1; }
  tail -1 $O/p$1_w$2.log | cut -c1-200
  python3 $R/tools/trace_crit.py $(find $O/p$1_w$2 -name "*.db" | head -1) | tee $O/p$1_w$2.crit
  find $O/p$1_w$2 -name "*.db" -delete
done
