#!/bin/bash
# Native distributed driver (bin/svdj_dist_main) vs the Python/torch solver
# (bench.py under torch.distributed.run), same sizes, ranks sharing one GPU
# over RCCL, one warmup solve each.  Output: gpurun_out/native_ab/.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/native_ab
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
E=svd-jacobi-mpi-cuda_amd/bin/svdj_dist_main
port=29700
for cfg in ${CFGS:-"1 16384" "2 4096" "2 8192" "4 8192"}; do
  set -- $cfg
  P=$1; N=$2
  sh=""; [ "$P" -gt 1 ] && sh="--shared-gpu"
  timeout -k 10 300 $E $N --np $P $sh --dtype f32 --input dense --warmup 1 > $O/native_p${P}_$N.log 2>&1 \
    || { echo "native P=$P N=$N failed"; tail -20 $O/native_p${P}_$N.log; exit 1; }
  echo "native P=$P N=$N: $(grep -E 'time with' $O/native_p${P}_$N.log) $(grep -oE 'sweeps: [0-9]+' $O/native_p${P}_$N.log)"
  port=$((port + 1))
  SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=nccl timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $P --master-addr 127.0.0.1 --master-port $port bench.py --gpus $P --size $N \
    --steps 1 --warmup 1 --no-verify --json-out $O/py_p${P}_$N.json > $O/py_p${P}_$N.log 2>&1 \
    || { echo "python P=$P N=$N failed"; tail -20 $O/py_p${P}_$N.log; exit 1; }
  echo "python P=$P N=$N: $(python3 -c "import json; d=json.load(open('$O/py_p${P}_$N.json')); print(d['ms_per_step'], d['sweeps'])")"
done
