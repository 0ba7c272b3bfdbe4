#!/bin/bash
# New apply workgroup rule (2048 WGs for >= 64 pairs per step, else 512) vs
# the old fixed 2048 (SVDJ_APPLY_WG_TARGET=2048) on the other configurations.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/awg3
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
run() {  # name, env value ("" = new rule), bench args
  local name=$1 t=$2; shift 2
  SVDJ_APPLY_WG_TARGET=$t timeout -k 10 300 python -u bench.py "$@" --json-out $O/$name.json > $O/$name.log 2>&1 \
    || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(python3 -c "import json; d=json.load(open('$O/$name.json')); print(d.get('ms_per_step', d.get('value')), d.get('sweeps'))")"
}
for v in new old; do
  t=""; [ $v = old ] && t=2048
  run f32_4096_$v "$t" --n 4096 --steps 3 --warmup 1
  run f32_8192_$v "$t" --n 8192 --steps 2 --warmup 1
  run tall_$v "$t" --n 8192 --m 32768 --steps 1 --warmup 1
  run f64_5000_$v "$t" --n 5000 --dtype fp64 --steps 1 --warmup 1
  run f64_16384_$v "$t" --n 16384 --dtype fp64 --steps 1 --warmup 0 --no-verify
  run sim8_$v "$t" --simulate-P 8 --n 16384 --sim-sweeps 2
done
