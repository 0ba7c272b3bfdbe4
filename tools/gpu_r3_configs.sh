# Round-3 config refresh with the split-bf16 default (dev aid): BASELINE config 5
# (65536^2 fp32, 1 GPU, to convergence) and the reference's fp64 job sizes.
set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
b() { tag=$1; t=$2; shift 2; timeout -k 10 $t python3 -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log > $O/$tag.json
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read());a=d.get('accuracy') or {};print(sys.argv[2],d['ms_per_step'],d['value'],d.get('sweeps'),d['config'].get('block_W'),d['config'].get('inner_order'),d['config'].get('mma'),'res',a.get('residual_rel'))" $O/$tag.json $tag; }
b f64_5000 200 --n 5000 --dtype fp64 --steps 3 --warmup 1
b f64_20000 300 --n 20000 --dtype fp64 --steps 1 --warmup 0 --no-verify
b f64_30000 400 --n 30000 --dtype fp64 --steps 1 --warmup 0 --no-verify
SW=3 bash tools/gpu_ab_sim.sh 16384 8 w32:"--block 32" && STEPS=3 bash tools/gpu_ab_args.sh 4096 w32:"--block 32"
