set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 "$@" > gpurun_out/tt_$tag.log 2>&1 || { tail -20 gpurun_out/tt_$tag.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/tt_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['sweeps'], d['config'].get('precondition'), d['config'].get('mma'), d['accuracy'], d['off_history_last'])"
}
run tall_fp32_qr --m 32768 --size 8192 --precondition qr && run tall_fp32_none --m 32768 --size 8192 --precondition none && run tall_bf16_qr --m 32768 --size 8192 --dtype bf16 --precondition qr
