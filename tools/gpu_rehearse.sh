# The driver's multi-GPU bench command rehearsed on ONE GPU (SVDJ_SHARED_GPU=1:
# all ranks on cuda:0 over RCCL's socket transport) with the production defaults.
# Usage: bash tools/gpu_rehearse.sh "2 4 8" SIZE ENGINE [extra bench args]
# Every rank-0 sweep prints a progress line, so a slow run is told from a hang.
set -o pipefail
NS=${1:-"2 4 8"}; SIZE=${2:-8192}; ENGINE=${3:-python}; shift 3 2>/dev/null
O=gpurun_out/rehearse; mkdir -p $O
for N in $NS; do
  L=$O/n${N}_${SIZE}_${ENGINE}.log
  SVDJ_SHARED_GPU=1 SVDJ_COMM_TIMEOUT=300 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N \
    --size $SIZE --steps 1 --warmup 0 --progress --engine $ENGINE "$@" > $L 2>&1 \
    || { echo "N=$N failed"; grep -v amdgpu.ids $L | tail -20; exit 1; }
  grep -c "sweep" $L | sed "s/^/N=$N progress lines: /"
  tail -1 $L | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('N',d['n_gpus'],'ms',d['ms_per_step'],'sweeps',d['sweeps'],'W',c['block_W'],c['mma'],c['inner_order'],c.get('exchange'),'res',(d.get('accuracy') or {}).get('residual_rel'),'world',d.get('world'),'comm',d.get('comm'))"
done
