#!/bin/bash
# bench.py through torch.distributed.run with RCCL ranks sharing the one GPU
# (the driver's multi-GPU command shape), 2 and 4 ranks.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/rccl_bench
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1 SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=nccl
port=29810
for cfg in ${CFGS:-2:8192 4:8192}; do
  set -- ${cfg/:/ }
  port=$((port + 1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $1 --size $2 --steps 1 --warmup 1 --json-out $O/p$1_$2.json \
    > $O/p$1_$2.log 2>&1 || { echo "P=$1 failed"; tail -30 $O/p$1_$2.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/p$1_$2.json')); print('P=$1 n=$2', d['ms_per_step'], d['sweeps'], d['config']['block_W'], d['comm'], d['accuracy'])"
done
