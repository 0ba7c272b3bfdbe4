#!/bin/bash
# hipGraph replay of the staggered two-chain issue (default) vs eager issue.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/graph
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_drivers.py tests/test_gpu_multirank.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in 1 0; do
  for n in 2048 4096 8192 16384; do
    SVDJ_GRAPH=$g timeout -k 10 300 python -u bench.py --n $n --steps 2 --warmup 1 --no-verify --json-out $O/g${g}_$n.json > $O/g${g}_$n.log 2>&1 || { tail -20 $O/g${g}_$n.log; exit 1; }
    echo "graph=$g n=$n: $(python3 -c "import json; d=json.load(open('$O/g${g}_$n.json')); print(d['ms_per_step'], d['sweeps'])")"
  done
  SVDJ_GRAPH=$g timeout -k 10 300 python -u bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 --json-out $O/g${g}_sim8.json > $O/g${g}_sim8.log 2>&1 || { tail -20 $O/g${g}_sim8.log; exit 1; }
  echo "graph=$g sim8: $(python3 -c "import json; print(json.load(open('$O/g${g}_sim8.json'))['value'])")"
done
