# Rehearse the 2-rank RCCL pipelined path on ONE GPU (both ranks on cuda:0).
set -o pipefail
export SVDJ_NO_AUTOBUILD=1 SVDJ_SHARED_GPU=1 SVDJ_COMM_BACKEND=${SVDJ_COMM_BACKEND:-gloo}
mkdir -p gpurun_out
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --size ${1:-2048} --steps 1 --warmup 1 ${@:2} > gpurun_out/shared2.log 2>&1
rc=$?; tail -25 gpurun_out/shared2.log; exit $rc
