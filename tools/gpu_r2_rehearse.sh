#!/bin/bash
# The driver's multi-GPU bench command (torch.distributed.run, bench.py
# --gpus N) rehearsed with N ranks sharing the one GPU over RCCL
# (SVDJ_SHARED_GPU=1): JSON contract, comm timing, accuracy at N = 2, 4, 8.
set -o pipefail
cd "$(dirname "$0")/.."
export SVDJ_NO_AUTOBUILD=1 SVDJ_SHARED_GPU=1
O=gpurun_out/rehearse
mkdir -p $O
for N in ${NS:-2 4 8}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps 1 --warmup 1 --size ${SIZE:-4096} \
    --json-out $O/n$N.json > $O/n$N.log 2>&1 || { tail -20 $O/n$N.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/n$N.json')); print('N=$N', d['ms_per_step'], 'ms', d['sweeps'], d['comm'], d['accuracy'])"
done
