#!/bin/bash
# EVD with Q rows on every wave (default) vs waves 1..15 (variant q15).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/qall
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in default q15; do
  lib=""; [ $v != default ] && lib=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_$v.so
  for cfg in 8:64 8:32 4:64; do
    set -- ${cfg/:/ }
    SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --block $2 --json-out $O/${v}_p$1_w$2.json > $O/${v}_p$1_w$2.log 2>&1 || { tail -20 $O/${v}_p$1_w$2.log; exit 1; }
    echo "$v sim P=$1 W=$2: $(python3 -c "import json; print(json.load(open('$O/${v}_p$1_w$2.json'))['value'])")"
  done
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --no-verify \
    --json-out $O/${v}_one.json > $O/${v}_one.log 2>&1 || { tail -20 $O/${v}_one.log; exit 1; }
  echo "$v 1-GPU 16384: $(python3 -c "import json; d=json.load(open('$O/${v}_one.json')); print(d['ms_per_step'], d['sweeps'])")"
done
SVDJ_HIP_LIB=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_prof.so timeout -k 10 120 python3 tools/evd_phase_profile.py --m 16384 --pairs 8 --cases fp32:64,fp32:32
