#!/bin/bash
# fp32 W=64 cross Gram rows per lane per slab: 8 (default) vs 16 vs 4.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/lpl
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in default lpl16 lpl4; do
  lib=""; [ $v != default ] && lib=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_$v.so
  SVDJ_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_iso -o run --output-format csv \
    -- python3 $R/tools/evd_ab.py --n 8192 --block 64 --sweeps 1 > $O/${v}_iso.log 2>&1 || { tail -20 $O/${v}_iso.log; exit 1; }
  python3 - $O/${v}_iso $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gram_kernel<float, 64, 0>" in r["Name"]:
            print("%-8s %-36s avg %8.1f us" % (sys.argv[2], r["Name"].split("(")[0][-36:], float(r["AverageNs"]) / 1e3))
PY
  cd $R
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --no-verify --json-out $O/one_$v.json > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 --json-out $O/sim8_$v.json > $O/sim8_$v.log 2>&1 || { tail -20 $O/sim8_$v.log; exit 1; }
  echo "$v: 1-GPU $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], d['sweeps'])") sim8 $(python3 -c "import json; print(json.load(open('$O/sim8_$v.json'))['value'])")"
  cd /tmp
done
