#!/bin/bash
# Per-rank plan of the 8-GPU 16384^2 job (simulated on one GPU): kernel-time
# breakdown (rocprofv3 stats), W=32 vs W=64, and the fp64 MFMA PMC pass.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out/simprof
export SVDJ_NO_AUTOBUILD=1
for W in 32 64; do
  timeout -k 10 300 python -u bench.py --simulate-P 8 --simulate-rank 0 --n 16384 --sim-sweeps 2 --block $W \
    > gpurun_out/simprof/sim_w$W.log 2>&1 || { tail -20 gpurun_out/simprof/sim_w$W.log; exit 1; }
  tail -1 gpurun_out/simprof/sim_w$W.log | cut -c 1-300
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/simprof/prof -o run --output-format csv \
  -- python $R/bench.py --simulate-P 8 --simulate-rank 0 --n 16384 --sim-sweeps 2 > $R/gpurun_out/simprof/prof.log 2>&1 \
  || { tail -20 $R/gpurun_out/simprof/prof.log; exit 1; }
python3 - $R/gpurun_out/simprof/prof <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:10]:
        print("   %-50s calls %7s total %9.1f ms avg %8.1f us" % (r["Name"].split("(")[0][-50:], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
cd $R
PMC_PASSES="1 2" PMC_CMD="python3 $R/tools/evd_ab.py --n 8192 --block 64 --dtype fp64 --sweeps 1" bash tools/gpu_pmc.sh pmc_fp64_w64 8192 > /dev/null && head -8 gpurun_out/pmc_fp64_w64/summary.md
