# A/B of chain issue modes at small sizes (dev aid).  Usage: bash tools/gpu_ab_small.sh "4096 8192"
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for N in ${1:-4096}; do
  for v in "default:" "stagger:--stagger" "chains1:--chains 1" "native:--engine native"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 200 python3 bench.py --n $N --steps 5 --warmup 2 --no-verify $args > gpurun_out/ab/${N}_$name.log 2>&1 || { tail -5 gpurun_out/ab/${N}_$name.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],d['ms_per_step'],d['sweeps'])" gpurun_out/ab/${N}_$name.log $N $name
  done
done
