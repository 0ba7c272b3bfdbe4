# Cross Gram variants (SVDJ_GRAM_VARIANT 0..3) on the single-stream step probe and the
# 16384^2 bench (dev aid).  Usage: bash tools/gpu_gram_variants.sh TAG "0 1 2 3" "0 3"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gramvar_$1; mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for v in $2; do
  SVDJ_GRAM_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/v$v -o run --output-format csv -- \
    python3 $R/tools/step_probe.py --no-copy --reps 2 > $O/probe_v$v.log 2>&1 || { tail -5 $O/probe_v$v.log; exit 1; }
  echo "v$v $(grep '"rep": 1' $O/probe_v$v.log | cut -c1-160)"
  python3 - $O/v$v/run_kernel_stats.csv <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if "gram" in x["Name"] or "apply" in x["Name"]:
        print("   %-50s %8.1f us" % (x["Name"][:50], float(x["AverageNs"]) / 1e3))
PY
done
for v in $3; do
  SVDJ_GRAM_VARIANT=$v timeout -k 10 300 python3 -u $R/bench.py --n 16384 --steps 1 --warmup 0 > $O/bench_v$v.log 2>&1 || { tail -5 $O/bench_v$v.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]);a=d['accuracy'];print('bench v$v',d['ms_per_step'],d['sweeps'],a['residual_rel'],a['orth_u_max_abs'],a['orth_v_max_abs'])" $O/bench_v$v.log
done
