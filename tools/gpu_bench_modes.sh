# bench.py per matrix-core mode with the accuracy check (dev aid).
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
N=${1:-16384}; MODES=${2:-"native bf16x6"}
mkdir -p gpurun_out
for mma in $MODES; do
  timeout -k 10 400 python bench.py --n $N --steps 1 --warmup 1 --mma $mma > gpurun_out/bm_${N}_$mma.log 2>&1 \
    || { tail -20 gpurun_out/bm_${N}_$mma.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bm_${N}_$mma.log').read().strip().splitlines()[-1]); print('$mma', d['value'], d['ms_per_step'], d['sweeps'], d['accuracy'])"
done
