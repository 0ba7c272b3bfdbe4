#!/bin/bash
# Apply X-tile prefetch depth 2 (variant lib -DSVDJ_APPLY_DEPTH=2) vs 1:
# kernel tests on the variant, rank plans, 1-GPU sizes.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/depth
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
V=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_depth2.so
SVDJ_HIP_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name lib args
  local name=$1 L=$2; shift 2
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py "$@" --json-out $O/$name.json > $O/$name.log 2>&1 \
    || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(python3 -c "import json; d=json.load(open('$O/$name.json')); print(d.get('ms_per_step', d.get('value')))")"
}
for v in d2 d1; do
  L=""; [ $v = d2 ] && L=$V
  run sim8_$v "$L" --simulate-P 8 --n 16384 --sim-sweeps 2
  run sim4_$v "$L" --simulate-P 4 --n 16384 --sim-sweeps 2
  run sim2_$v "$L" --simulate-P 2 --n 16384 --sim-sweeps 2
  run one16k_$v "$L" --n 16384 --steps 2 --warmup 1
  run one4k_$v "$L" --n 4096 --steps 3 --warmup 1
  run f64_5000_$v "$L" --n 5000 --dtype fp64 --steps 1 --warmup 1
done
