#!/bin/bash
# A/B of the apply's 16-byte Q fill (default) vs the element-wise fill
# (variant lib, -DSVDJ_APPLY_Q16=0) on the 4- and 8-GPU rank plans, twice.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/q16
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for rep in 1 2; do
  for v in on off; do
    L=""; [ $v = off ] && L=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_q16off.so
    for P in 4 8; do
      SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --sim-sweeps 2 \
        --json-out $O/p${P}_${v}_$rep.json > $O/p${P}_${v}_$rep.log 2>&1 || { tail -20 $O/p${P}_${v}_$rep.log; exit 1; }
      echo "q16=$v P=$P rep $rep: $(python3 -c "import json; print(json.load(open('$O/p${P}_${v}_$rep.json'))['value'])")"
    done
  done
done
