# Round-3 final measurements with the split-bf16 default (dev aid): headline and
# config benches, rank-plan simulations, one PMC set on the 1-GPU headline.
set -o pipefail
O=gpurun_out/r3f; mkdir -p $O
b() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json.log 2>&1 || { tail -5 $O/$tag.json.log; exit 1; }
  tail -1 $O/$tag.json.log > $O/$tag.json
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read());a=d.get('accuracy') or {};print(sys.argv[2],d['ms_per_step'],d['value'],d.get('sweeps'),'res',a.get('residual_rel'),'sig',a.get('sigma_max_rel_err_vs_fp64_oracle'))" $O/$tag.json $tag; }
b headline16384 --steps 3 --warmup 1
b n4096 --n 4096 --steps 5 --warmup 2 --check-sigma
b n8192 --n 8192 --steps 3 --warmup 1 --check-sigma
b tall_fp32 --m 32768 --n 8192 --steps 3 --warmup 1
b tall_bf16 --m 32768 --n 8192 --dtype bf16 --steps 3 --warmup 1
b f64_10000 --n 10000 --dtype fp64 --steps 2 --warmup 1
for P in 8 4 2 1; do b sim$P --simulate-P $P --n 16384 --sim-sweeps 3; done
b sim8_g100 --simulate-P 8 --n 16384 --sim-sweeps 3 --sim-link-gbps 100
b sim8_g50 --simulate-P 8 --n 16384 --sim-sweeps 3 --sim-link-gbps 50
PMC_PASSES="1 3 4" bash tools/gpu_pmc.sh r3f/pmc 16384 || exit 1
head -6 $O/pmc/summary.md
