# Generic bench A/B (dev aid).  Usage: bash tools/gpu_ab_args.sh N "name:args" ["name:args" ...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
N=$1; shift
for v in "$@"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python3 bench.py --n $N --steps ${STEPS:-5} --warmup 2 --no-verify $args > gpurun_out/ab/${N}_$name.log 2>&1 || { tail -5 gpurun_out/ab/${N}_$name.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],d['ms_per_step'],d['sweeps'],d['config']['block_W'],d['config']['inner_order'])" gpurun_out/ab/${N}_$name.log $N $name
done
