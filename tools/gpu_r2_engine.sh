#!/bin/bash
# bench.py --engine native (libsvdj_dist inside the bench process) vs the
# Python executor: 1 GPU at 16384^2, then 2 and 4 ranks sharing the GPU over
# RCCL (torch.distributed.run) at 8192^2.  Output: gpurun_out/engine/.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/engine
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
for e in native python; do
  timeout -k 10 300 python -u bench.py --engine $e --size ${N1:-16384} --steps 1 --warmup 1 --progress \
    --json-out $O/one_$e.json > $O/one_$e.log 2>&1 || { echo "$e 1-GPU failed"; tail -20 $O/one_$e.log; exit 1; }
  echo "$e 1 GPU: $(python3 -c "import json; d=json.load(open('$O/one_$e.json')); print(d['ms_per_step'], 'ms', d['sweeps'], d['accuracy'])")"
done
port=29810
for P in ${PS:-2 4}; do
  for e in native python; do
    port=$((port + 1))
    SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=nccl timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $P --master-addr 127.0.0.1 --master-port $port bench.py --gpus $P --engine $e \
      --size ${N2:-8192} --steps 1 --warmup 1 --json-out $O/p${P}_$e.json > $O/p${P}_$e.log 2>&1 \
      || { echo "$e P=$P failed"; tail -30 $O/p${P}_$e.log; exit 1; }
    echo "$e P=$P: $(python3 -c "import json; d=json.load(open('$O/p${P}_$e.json')); print(d['ms_per_step'], 'ms', d['sweeps'], d['accuracy'])")"
  done
done
