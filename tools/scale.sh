#!/bin/bash
# Strong-scaling run of the headline benchmark on ONE node: N = 1, 2, 4, 8
# GPUs, one process per GPU (torchrun, RCCL), one JSON line per N written to
# OUT/scale_nN.json.  The reference's job scripts ran 2 ranks
# (build/runSVDMPICUDA.slurm:4-7, 24-26); this sweeps the whole node.
# Usage: bash tools/scale.sh [OUT=gpurun_out/scale] [extra bench.py args]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/scale}; shift || true
mkdir -p "$OUT"
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
for N in 1 2 4 8; do
  if [ "$N" -gt "$NGPU" ]; then echo "skip N=$N (only $NGPU GPUs)"; continue; fi
  PORT=$((29500 + N))
  if [ "$N" -eq 1 ]; then
    CMD=(python3 bench.py --gpus 1)
  else
    CMD=(python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1
         --master-port "$PORT" bench.py --gpus "$N")
  fi
  SVDJ_COMM_TIMEOUT=${SVDJ_COMM_TIMEOUT:-300} timeout -k 10 1200 "${CMD[@]}" --json-out "$OUT/scale_n$N.json" "$@" \
    > "$OUT/scale_n$N.log" 2>&1 || { echo "N=$N failed"; tail -20 "$OUT/scale_n$N.log"; exit 1; }
  tail -1 "$OUT/scale_n$N.log"
done
