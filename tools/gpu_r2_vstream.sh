#!/bin/bash
# Deferred V rotation on a side stream per chain (SVDJ_VSTREAM=1) vs inline,
# with 4 and 8 hardware queues per process.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/vstream
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
SVDJ_VSTREAM=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_drivers.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for q in 4 8; do
  for vs in 0 1; do
    for cfg in 8:64 4:64 2:64; do
      set -- ${cfg/:/ }
      GPU_MAX_HW_QUEUES=$q SVDJ_VSTREAM=$vs timeout -k 10 300 python -u bench.py --simulate-P $1 --n 16384 --sim-sweeps 2 \
        --block $2 --json-out $O/q${q}_v${vs}_p$1.json > $O/q${q}_v${vs}_p$1.log 2>&1 || { tail -20 $O/q${q}_v${vs}_p$1.log; exit 1; }
      echo "queues=$q vstream=$vs P=$1: $(python3 -c "import json; print(json.load(open('$O/q${q}_v${vs}_p$1.json'))['value'])")"
    done
    GPU_MAX_HW_QUEUES=$q SVDJ_VSTREAM=$vs timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --no-verify \
      --json-out $O/q${q}_v${vs}_one.json > $O/q${q}_v${vs}_one.log 2>&1 || { tail -20 $O/q${q}_v${vs}_one.log; exit 1; }
    echo "queues=$q vstream=$vs 1-GPU: $(python3 -c "import json; d=json.load(open('$O/q${q}_v${vs}_one.json')); print(d['ms_per_step'], d['sweeps'])")"
  done
done
