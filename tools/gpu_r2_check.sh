#!/bin/bash
# Quick regression check after a kernel/geometry change: kernel tests, the
# 8-GPU rank plans, a few one-GPU solves (fp32 / fp64).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/check
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in ${SIMS:-8:32 8:64 4:64 2:64}; do
  set -- ${cfg/:/ }
  timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 --sim-sweeps 2 --block $2 \
    --json-out $O/sim_p$1_w$2.json > $O/sim_p$1_w$2.log 2>&1 || { tail -20 $O/sim_p$1_w$2.log; exit 1; }
  echo "sim P=$1 W=$2: $(python3 -c "import json; print(json.load(open('$O/sim_p$1_w$2.json'))['value'])") ms/sweep"
done
for cfg in ${ONES:-4096:fp32 16384:fp32 5000:fp64}; do
  set -- ${cfg/:/ }
  timeout -k 10 300 python -u bench.py --n $1 --dtype $2 --steps 1 --warmup 1 --json-out $O/one_$1_$2.json \
    > $O/one_$1_$2.log 2>&1 || { tail -20 $O/one_$1_$2.log; exit 1; }
  echo "1-GPU $1 $2: $(python3 -c "import json; d=json.load(open('$O/one_$1_$2.json')); print(d['ms_per_step'], 'ms', d['sweeps'], d['config']['block_W'], d['accuracy']['residual_rel'])")"
done
