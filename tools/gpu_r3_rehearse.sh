# The driver's multi-GPU bench command at N = 2, 4, 8 rehearsed on ONE GPU
# (SVDJ_SHARED_GPU=1: all ranks on cuda:0 over RCCL's socket transport), with
# the round-3 defaults (split-bf16 apply, cross EVD) at 8192^2 (dev aid).
set -o pipefail
O=gpurun_out/rehearse; mkdir -p $O
for N in 2 4 8; do
  SVDJ_SHARED_GPU=1 SVDJ_COMM_TIMEOUT=300 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N \
    --size 8192 --steps 1 --warmup 1 > $O/n$N.log 2>&1 || { echo "N=$N failed"; tail -20 $O/n$N.log; exit 1; }
  tail -1 $O/n$N.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('N',d['n_gpus'],d['ms_per_step'],d['sweeps'],c['block_W'],c['mma'],c['inner_order'],(d.get('accuracy') or {}).get('residual_rel'),d.get('world'),d.get('devices'))"
done
