#!/bin/bash
# Kernel traces of simulated rank plans (16384^2 fp32): P=2 W=64, P=8 W=32.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/simtrace
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-2:64 8:32}; do   # P:W
  set -- ${cfg/:/ }
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$1_w$2 -o run -- python $R/bench.py --simulate-P $1 \
    --simulate-rank 0 --n ${N:-16384} --sim-sweeps 2 --block $2 > $O/p$1_w$2.log 2>&1 || { tail -20 $O/p$1_w$2.log; exit 1; }
  python3 $R/tools/trace_db_summary.py $(find $O/p$1_w$2 -name "*.db" | head -1)
done
