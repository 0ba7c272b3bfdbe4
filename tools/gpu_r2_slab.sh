#!/bin/bash
# EVD slab-sum loads in flight (SVDJ_EVD_SLAB_UNROLL 16 default vs 8 / 32
# variant libs): kernel tests, rank plans P=8/4, 1-GPU 16384^2.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/slab
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 16 8 32; do
  L=""; [ $v != 16 ] && L=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_slab$v.so
  for P in 8 4; do
    SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --json-out $O/p${P}_u$v.json > $O/p${P}_u$v.log 2>&1 || { tail -20 $O/p${P}_u$v.log; exit 1; }
    echo "unroll=$v P=$P: $(python3 -c "import json; print(json.load(open('$O/p${P}_u$v.json'))['value'])")"
  done
done
