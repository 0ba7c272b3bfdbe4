#!/bin/bash
# Bipartite vs cyclic EVD ordering of the cross steps: kernel tests, isolated
# EVD latency, simulated rank plans (16384^2 fp32 at P = 2, 8) and the 1-GPU
# headline solve to convergence.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/bip
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "bipartite or matches_reference or end_to_end" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for ord in cyclic bipartite; do
  for cfg in ${SIMS:-"8 32" "8 64" "2 64"}; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --simulate-P $1 --simulate-rank 0 --n 16384 --sim-sweeps 2 --block $2 \
      --inner-order $ord --json-out $O/sim_p$1_w$2_$ord.json > $O/sim_p$1_w$2_$ord.log 2>&1 || { tail -20 $O/sim_p$1_w$2_$ord.log; exit 1; }
    echo "$ord sim P=$1 W=$2: $(python3 -c "import json; print(json.load(open('$O/sim_p$1_w$2_$ord.json'))['value'])") ms/sweep"
  done
done
for ord in cyclic bipartite; do
  for n in ${SIZES:-4096 16384}; do
    timeout -k 10 300 python -u bench.py --n $n --steps 1 --warmup 1 --inner-order $ord --json-out $O/bench_${n}_$ord.json \
      > $O/bench_${n}_$ord.log 2>&1 || { tail -20 $O/bench_${n}_$ord.log; exit 1; }
    echo "$ord 1-GPU n=$n: $(python3 -c "import json; d=json.load(open('$O/bench_${n}_$ord.json')); print(d['ms_per_step'], 'ms', d['sweeps'], 'sweeps', d['accuracy'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for ord in cyclic bipartite; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/iso_$ord -o run --output-format csv \
    -- python3 $R/bench.py --simulate-P 8 --simulate-rank 0 --n 16384 --sim-sweeps 1 --inner-order $ord > $O/iso_$ord.log 2>&1 || { tail -20 $O/iso_$ord.log; exit 1; }
  python3 - $O/iso_$ord $ord <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:5]:
        print("  %-10s %-45s calls %6s avg %8.1f us" % (sys.argv[2], r["Name"].split("(")[0][-45:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
