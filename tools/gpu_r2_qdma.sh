#!/bin/bash
# Apply Q fill by LDS-DMA (variant lib -DSVDJ_APPLY_Q16=2) vs element-wise
# (default): kernel tests on the variant, rank plans, 1-GPU 16384^2.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/qdma
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
V=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_qdma.so
SVDJ_HIP_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in dma def; do
  L=""; [ $v = dma ] && L=$V
  for P in 8 4 2; do
    SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --json-out $O/p${P}_${v}_$rep.json > $O/p${P}_${v}_$rep.log 2>&1 || { tail -20 $O/p${P}_${v}_$rep.log; exit 1; }
    echo "$v P=$P rep $rep: $(python3 -c "import json; print(json.load(open('$O/p${P}_${v}_$rep.json'))['value'])")"
  done
done
done
for v in dma def; do
  L=""; [ $v = dma ] && L=$V
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 --json-out $O/one_$v.json \
    > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  echo "$v 1-GPU: $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], d['sweeps'], d['accuracy']['residual_rel'])")"
done
