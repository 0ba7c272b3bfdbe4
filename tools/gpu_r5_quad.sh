#!/bin/bash
# Round-5 quad-step evaluation on one MI355X: GPU quad tests, headline size
# with quad on/off, smaller sizes, rank-plan simulations.  Every step under its
# own time limit; progress goes to files under gpurun_out/ as it runs.
set -o pipefail
D=${1:-gpurun_out/r5e}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_quad.py -v --timeout 200 --timeout-method thread > $D/pytest_quad.log 2>&1
echo "pytest rc=$?" | tee -a $D/summary.txt
for Q in on off; do
  for N in 16384 8192 4096; do
    timeout -k 10 300 python -u bench.py --n $N --steps 2 --warmup 1 --quad $Q --progress --json-out $D/bench_${N}_$Q.json > $D/bench_${N}_$Q.log 2>&1 || { echo "bench $N $Q failed" | tee -a $D/summary.txt; exit 1; }
  done
done
for P in 2 4 8; do
  for Q in on off; do
    timeout -k 10 300 python -u bench.py --n 16384 --simulate-P $P --sim-sweeps 3 --quad $Q --json-out $D/sim${P}_$Q.json > $D/sim${P}_$Q.log 2>&1 || { echo "sim $P $Q failed" | tee -a $D/summary.txt; exit 1; }
  done
done
python - $D <<'PY' | tee -a $D/summary.txt
import json, sys, glob, os
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    j = json.load(open(f))
    acc = j.get("accuracy") or {}
    print(os.path.basename(f), j.get("value"), j.get("unit"), j.get("ms_per_step", j.get("solve_s")),
          j.get("sweeps", j.get("sweeps_run")), acc.get("residual_rel"), acc.get("orth_u_max_abs"),
          acc.get("orth_v_max_abs"), acc.get("sigma_max_rel_err_vs_fp64_oracle"))
PY
