# Spread (all-link, relayed) vs direct exchange: RCCL multi-rank tests on one
# GPU, then simulated rank plans of 16384^2 fp32 with modelled link speeds.
# Usage (via gpurun): bash tools/gpu_spread.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/spread
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 \
  --timeout-method thread > $O/pytest_multirank.log 2>&1 || { tail -30 $O/pytest_multirank.log; exit 1; }
tail -3 $O/pytest_multirank.log
for P in 8 4; do for g in 100 50; do for ex in direct spread; do
  timeout -k 10 200 python bench.py --simulate-P $P --n 16384 --sim-sweeps 2 --sim-link-gbps $g \
    --exchange $ex > $O/sim${P}_g${g}_$ex.json 2> $O/sim.err || { tail $O/sim.err; exit 1; }
  echo "P=$P link=$g $ex $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['comm'].get('exposed_comm_ms'))" $O/sim${P}_g${g}_$ex.json)"
done; done; done
