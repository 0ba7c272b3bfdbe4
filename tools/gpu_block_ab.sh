# bench.py with W=32 vs W=64 per size (dev aid): tools/gpu_block_ab.sh "4096 8192"
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out
for N in ${1:-4096 8192}; do
  for W in 32 64; do
    timeout -k 10 300 python bench.py --n $N --steps 1 --warmup 1 --block $W ${EXTRA:-} \
      > gpurun_out/bw_${N}_$W.log 2>&1 || { tail -20 gpurun_out/bw_${N}_$W.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bw_${N}_$W.log').read().strip().splitlines()[-1]); print('n=$N W=$W', d['value'], d['ms_per_step'], d['sweeps'], d['accuracy']['residual_rel'])"
  done
done
