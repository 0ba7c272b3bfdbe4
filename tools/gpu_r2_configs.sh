#!/bin/bash
# BASELINE configs on one GPU: fp64 at the reference's job sizes (n = 5000,
# 10000, 20000, 30000; build/runSVDMPICUDAWithoutCMake.slurm:30-33) and 16384,
# the tall bf16 config (QR path) 4-GPU per-rank simulation.  STEP selects a subset.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/cfg
export SVDJ_NO_AUTOBUILD=1
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  if [ -n "$STEP" ] && ! [[ " $STEP " == *" $name "* ]]; then return 0; fi
  timeout -k 10 $to python -u bench.py "$@" --json-out gpurun_out/cfg/$name.json > gpurun_out/cfg/$name.log 2>&1 \
    || { echo "$name failed"; tail -20 gpurun_out/cfg/$name.log; exit 1; }
  echo "== $name"; tail -1 gpurun_out/cfg/$name.log
}
run sim_tall_bf16_p4 300 --n 8192 --m 32768 --dtype bf16 --simulate-P 4 --sim-sweeps 3
run fp64_5000 300 --n 5000 --dtype fp64 --steps 1 --warmup 1
run fp64_10000 400 --n 10000 --dtype fp64 --steps 1 --warmup 0
run fp64_16384 600 --n 16384 --dtype fp64 --steps 1 --warmup 0 --no-verify
run fp64_20000 900 --n 20000 --dtype fp64 --steps 1 --warmup 0 --no-verify --progress
run fp64_30000 1100 --n 30000 --dtype fp64 --steps 1 --warmup 0 --no-verify --progress
# BASELINE config 5 (65536^2 fp32) feasibility: two sweeps on one GPU, and one
# full-work sweep of rank 0's plan in the 8-GPU job
run big65536_2sweeps 900 --n 65536 --dtype fp32 --steps 1 --warmup 0 --no-verify --max-sweeps 2 --progress
run sim_big65536_p8 900 --n 65536 --dtype fp32 --simulate-P 8 --sim-sweeps 1
