# A/B of the quad-step kernels against a base build (development aid).
# Usage: bash tools/gpu_ab_quad.sh TAG [BASE_SO]
#   1. the quad-step GPU tests on the in-tree build;
#   2. per build (new, base): kernel-trace of tools/step_probe.py --quad (per-kernel us),
#      then one 16384^2 bench solve with its accuracy block.
# Logs under gpurun_out/abq_TAG/.  Every GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}; BASE=${2:-tools/ab/libsvdj_hip_base.so}
O=$R/gpurun_out/abq_$TAG
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in new base; do
  if [ $v = base ]; then export SVDJ_HIP_LIB=$R/$BASE; else unset SVDJ_HIP_LIB; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
    python3 -u $R/tools/step_probe.py --quad --pairs 128 --steps 24 --no-copy > $O/probe_$v.log 2>&1 \
    || { tail -20 $O/probe_$v.log; exit 1; }
  grep steps $O/probe_$v.log | tail -1
  python3 - $O/prof_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("  %-44s %6s %9.1f ms %8.1f us" % (x['Name'][:44], x['Calls'], float(x['TotalDurationNs'])/1e6, float(x['AverageNs'])/1e3))
PY
  timeout -k 10 300 python3 -u $R/bench.py --n 16384 --steps 2 --warmup 1 > $O/bench_$v.log 2>&1 \
    || { tail -20 $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['sweeps'], d['accuracy'])"
done
