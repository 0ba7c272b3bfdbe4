#!/bin/bash
# Apply Q-fragment prefetch distance (SVDJ_APPLY_QPD 8 default vs 4 / 16
# variant libs): 1-GPU 16384^2 and the 8-GPU rank plan.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/qpd
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for v in 8 4 16; do
  L=""; [ $v != 8 ] && L=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_qpd$v.so
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 \
    --json-out $O/p8_q$v.json > $O/p8_q$v.log 2>&1 || { tail -20 $O/p8_q$v.log; exit 1; }
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 \
    --json-out $O/one_q$v.json > $O/one_q$v.log 2>&1 || { tail -20 $O/one_q$v.log; exit 1; }
  echo "QPD=$v: P=8 $(python3 -c "import json; print(json.load(open('$O/p8_q$v.json'))['value'])") ms/sweep, 1-GPU $(python3 -c "import json; d=json.load(open('$O/one_q$v.json')); print(d['ms_per_step'], d['accuracy']['residual_rel'])")"
done
