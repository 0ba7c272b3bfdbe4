#!/bin/bash
# README measured table (one MI355X, to convergence, one warmup solve where it
# is cheap): fp32 sizes, tall QR cases, the reference's fp64 job sizes, the
# 65536^2 two-sweep check and the simulated 8-GPU rank plans.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/table
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
run() {  # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" --json-out $O/$name.json > $O/$name.log 2>&1 \
    || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(python3 -c "import json; d=json.load(open('$O/$name.json')); print(d.get('ms_per_step', d.get('value')), d.get('sweeps'), d.get('config', {}).get('block_W'), (d.get('accuracy') or {}).get('residual_rel'))")"
}
for spec in ${ROWS:-fp32_4096 fp32_8192 fp32_16384 tall_fp32 tall_bf16 fp64_5000 fp64_10000 fp64_16384 fp64_20000 fp64_30000 big65536 sim8 sim4 sim2}; do
  case $spec in
    fp32_4096) run $spec 200 --n 4096 --steps 2 --warmup 1 ;;
    fp32_8192) run $spec 200 --n 8192 --steps 2 --warmup 1 ;;
    fp32_16384) run $spec 300 --n 16384 --steps 2 --warmup 1 ;;
    tall_fp32) run $spec 200 --n 8192 --m 32768 --steps 1 --warmup 1 ;;
    tall_bf16) run $spec 200 --n 8192 --m 32768 --dtype bf16 --steps 1 --warmup 1 ;;
    fp64_5000) run $spec 200 --n 5000 --dtype fp64 --steps 1 --warmup 1 ;;
    fp64_10000) run $spec 200 --n 10000 --dtype fp64 --steps 1 --warmup 0 ;;
    fp64_16384) run $spec 300 --n 16384 --dtype fp64 --steps 1 --warmup 0 --no-verify ;;
    fp64_20000) run $spec 400 --n 20000 --dtype fp64 --steps 1 --warmup 0 --no-verify ;;
    fp64_30000) run $spec 600 --n 30000 --dtype fp64 --steps 1 --warmup 0 --no-verify ;;
    big65536) run $spec 400 --n 65536 --steps 1 --warmup 0 --max-sweeps 2 --no-verify ;;
    sim8) run $spec 200 --simulate-P 8 --n 16384 --sim-sweeps 2 ;;
    sim4) run $spec 200 --simulate-P 4 --n 16384 --sim-sweeps 2 ;;
    sim2) run $spec 200 --simulate-P 2 --n 16384 --sim-sweeps 2 ;;
  esac
done
