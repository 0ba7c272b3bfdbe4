# BASELINE.json configs that fit one GPU (dev aid): bench lines per config.
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/cfg_$tag.log 2>&1 || { tail -20 gpurun_out/cfg_$tag.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cfg_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['sweeps'], d['config'].get('precondition'), d['accuracy'])"
}
run n16384 --steps 1 --warmup 1 && run n4096 --size 4096 --steps 2 --warmup 1 && \
run tall_bf16 --m 32768 --size 8192 --dtype bf16 --steps 1 --warmup 1 && \
run tall_fp32_noqr --m 32768 --size 8192 --precondition none --steps 1 --warmup 0
