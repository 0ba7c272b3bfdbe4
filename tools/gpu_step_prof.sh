# rocprofv3 kernel stats of tools/step_probe.py (single stream), single and quad steps.
# Usage: bash tools/gpu_step_prof.sh TAG [probe args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift; EXTRA="$@"
O=$R/gpurun_out/stepprof_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp SVDJ_NO_AUTOBUILD=1
for v in single quad; do
  F=""; [ $v = quad ] && F="--quad"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
    python3 $R/tools/step_probe.py --no-copy --reps 2 $F $EXTRA > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep steps $O/$v.log
  python3 - $O/$v/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print("  %-56s %6s %9.2f ms %8.1f us" % (x['Name'][:56], x['Calls'], float(x['TotalDurationNs'])/1e6, float(x['AverageNs'])/1e3))
PY
done
