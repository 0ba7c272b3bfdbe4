#!/bin/bash
# Round-2 GPU check: RCCL multi-rank on one GPU (bitwise vs gloo), then the
# per-rank simulation of the 8-GPU 16384^2 plan.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 400 \
  --timeout-method thread > gpurun_out/mr.log 2>&1 || { tail -50 gpurun_out/mr.log; exit 1; }
tail -15 gpurun_out/mr.log
for P in 8 4 2; do
  timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 \
    --sim-sweeps 2 --json-out gpurun_out/sim_p$P.json > gpurun_out/sim_p$P.log 2>&1 \
    || { tail -30 gpurun_out/sim_p$P.log; exit 1; }
  tail -1 gpurun_out/sim_p$P.log
done
