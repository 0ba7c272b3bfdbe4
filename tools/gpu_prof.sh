# Kernel-time profile of one bench solve per matrix-core mode (dev aid).
# Usage: bash tools/gpu_prof.sh N "native bf16x6" [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-16384}; MODES=${2:-"native bf16x6"}; shift 2; EXTRA="$@"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for mma in $MODES; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${N}_$mma -o run \
    --output-format csv -- python $R/bench.py --n $N --steps 1 --warmup 0 --mma $mma $EXTRA \
    > $R/gpurun_out/prof_${N}_$mma.log 2>&1 || { tail -20 $R/gpurun_out/prof_${N}_$mma.log; exit 1; }
  tail -1 $R/gpurun_out/prof_${N}_$mma.log | cut -c1-300
  python - $R/gpurun_out/prof_${N}_$mma/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print("  %-48s %6s %9.1f ms %8.1f us" % (x['Name'][:48], x['Calls'], float(x['TotalDurationNs'])/1e6, float(x['AverageNs'])/1e3))
PY
done
