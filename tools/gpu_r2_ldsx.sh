#!/bin/bash
# fp32 apply with X staged in LDS (SVDJ_APPLY_LDSX=1) vs the default apply:
# GPU tests with it on, isolated apply timing under rocprofv3 (evd_ab.py), the
# simulated P=8 rank plan and the 1-GPU 16384^2 solve.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/ldsx
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
SVDJ_APPLY_LDSX=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py ${TESTS_EXTRA:-} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  for cfg in 4096:32 8192:64; do
    set -- ${cfg/:/ }
    SVDJ_APPLY_LDSX=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/l${v}_$1 -o run --output-format csv \
      -- python3 $R/tools/evd_ab.py --n $1 --block $2 > $O/l${v}_$1.log 2>&1 || { tail -20 $O/l${v}_$1.log; exit 1; }
    python3 - $O/l${v}_$1 $v $1 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "apply" in r["Name"]:
            print("ldsx=%s n=%s %-40s avg %8.1f us" % (sys.argv[2], sys.argv[3], r["Name"].split("(")[0][-40:], float(r["AverageNs"]) / 1e3))
PY
  done
done
cd $R
for v in 0 1; do
  SVDJ_APPLY_LDSX=$v timeout -k 10 300 python3 bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 \
    --json-out $O/sim8_$v.json > $O/sim8_$v.log 2>&1 || { tail -20 $O/sim8_$v.log; exit 1; }
  echo "ldsx=$v sim P=8: $(python3 -c "import json; print(json.load(open('$O/sim8_$v.json'))['value'])") ms/sweep"
  SVDJ_APPLY_LDSX=$v timeout -k 10 300 python3 bench.py --n 16384 --steps 1 --warmup 1 --no-verify \
    --json-out $O/one_$v.json > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  echo "ldsx=$v 1-GPU: $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], d['sweeps'])")"
done
