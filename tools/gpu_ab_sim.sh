# Rank-plan simulation A/B (dev aid).  Usage: bash tools/gpu_ab_sim.sh N P "name:args" ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
N=$1; P=$2; shift 2
for v in "$@"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python3 bench.py --simulate-P $P --n $N --sim-sweeps ${SW:-3} $args > gpurun_out/ab/sim${P}_${N}_$name.log 2>&1 || { tail -5 gpurun_out/ab/sim${P}_${N}_$name.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('sim',sys.argv[4],sys.argv[2],sys.argv[3],d['value'],d['config']['block_W'],d['config']['inner_order'])" gpurun_out/ab/sim${P}_${N}_$name.log $N $name $P
done
