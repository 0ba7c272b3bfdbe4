# bench.py per chain count (dev aid): tools/gpu_chains.sh N "2 4"
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
N=${1:-16384}; CH=${2:-"2 4"}
mkdir -p gpurun_out
for c in $CH; do
  timeout -k 10 400 python bench.py --n $N --steps 1 --warmup 1 --chains $c > gpurun_out/ch_${N}_$c.log 2>&1 \
    || { tail -20 gpurun_out/ch_${N}_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ch_${N}_$c.log').read().strip().splitlines()[-1]); print('chains $c', d['value'], d['ms_per_step'], d['sweeps'], d['accuracy'])"
done
