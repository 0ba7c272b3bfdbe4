#!/bin/bash
# sigma vs an fp64 oracle (fp32 and fp64 at <= 8192), root-owned end-to-end
# timing on one GPU and over two RCCL ranks sharing the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/misc
export SVDJ_NO_AUTOBUILD=1
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" --json-out gpurun_out/misc/$name.json > gpurun_out/misc/$name.log 2>&1 \
    || { echo "$name failed"; tail -20 gpurun_out/misc/$name.log; exit 1; }
  echo "== $name"; python3 -c "import json; d=json.load(open('gpurun_out/misc/$name.json')); print(d['n_gpus'], d['ms_per_step'], d['sweeps'], d['accuracy'], d.get('comm'))"
}
#run sigma_fp64_4096 python -u bench.py --n 4096 --dtype fp64 --steps 1 --warmup 1 --check-sigma
#run sigma_fp64_8192 python -u bench.py --n 8192 --dtype fp64 --steps 1 --warmup 0 --check-sigma
#run sigma_fp32_8192 python -u bench.py --n 8192 --dtype fp32 --steps 1 --warmup 1 --check-sigma
#run root_fp32_8192 python -u bench.py --n 8192 --steps 1 --warmup 1 --root-owned
SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=nccl run root_rccl2_4096 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --size 4096 --steps 1 --warmup 1 --root-owned
SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=nccl run otf_rccl2_4096 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --size 4096 --steps 1 --warmup 1 --check-sigma
