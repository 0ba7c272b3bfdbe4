set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out
for n in 8192 16384; do for inner in 2 3; do
  timeout -k 10 300 python bench.py --size $n --steps 1 --warmup 1 --inner $inner > gpurun_out/inner_${n}_$inner.log 2>&1 || { tail -5 gpurun_out/inner_${n}_$inner.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/inner_${n}_$inner.log').read().strip().splitlines()[-1]); print($n, 'inner', $inner, d['ms_per_step'], d['sweeps'], d['accuracy']['residual_rel'])"
done; done
