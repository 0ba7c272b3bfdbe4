#!/bin/bash
# Apply with Q in fragment order (one 16-byte LDS read per 4 / 2 MFMAs).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/qfrag
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
VLIB=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_qfrag.so
SVDJ_HIP_LIB=$VLIB timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in default qfrag; do
  lib=""; [ $v != default ] && lib=$VLIB
  for cfg in 4096:32:fp32 8192:64:fp32 4096:32:fp64 8192:64:fp64; do
    set -- ${cfg//:/ }
    SVDJ_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$1_$3 -o run --output-format csv \
      -- python3 $R/tools/evd_ab.py --n $1 --block $2 --dtype $3 --sweeps 1 > $O/${v}_$1_$3.log 2>&1 || { tail -20 $O/${v}_$1_$3.log; exit 1; }
    python3 - $O/${v}_$1_$3 $v $1 $3 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "apply" in r["Name"]:
            print("%-8s n=%s %s %-36s avg %8.1f us" % (sys.argv[2], sys.argv[3], sys.argv[4], r["Name"].split("(")[0][-36:], float(r["AverageNs"]) / 1e3))
PY
  done
done
cd $R
for v in default qfrag; do
  lib=""; [ $v != default ] && lib=$VLIB
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --no-verify --json-out $O/one_$v.json > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 --json-out $O/sim8_$v.json > $O/sim8_$v.log 2>&1 || { tail -20 $O/sim8_$v.log; exit 1; }
  echo "$v: 1-GPU $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], d['sweeps'])") sim8 $(python3 -c "import json; print(json.load(open('$O/sim8_$v.json'))['value'])")"
done
