#!/bin/bash
# Four chains (quarters) vs two (halves) on the simulated rank plans, with
# 4 and 8 hardware queues per process.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/chains4
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "multi_chain" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for q in ${QS:-4 8}; do
  for cfg in ${CFGS:-8:64:2 8:64:4 8:32:2 8:32:4 4:64:2 4:64:4 2:64:4}; do
    set -- ${cfg//:/ }
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --block $2 --chains $3 --json-out $O/q${q}_p$1_w$2_c$3.json > $O/q${q}_p$1_w$2_c$3.log 2>&1 || { tail -20 $O/q${q}_p$1_w$2_c$3.log; exit 1; }
    echo "queues=$q P=$1 W=$2 chains=$3: $(python3 -c "import json; print(json.load(open('$O/q${q}_p$1_w$2_c$3.json'))['value'])")"
  done
done
