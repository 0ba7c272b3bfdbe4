#!/bin/bash
# Apply-kernel variants (lib/variants/libsvdj_hip_<name>.so): isolated
# single-stream sweep timing under rocprofv3 (evd_ab.py) and the simulated
# P=8 rank plan of the 16384^2 job.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/apply_ab
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for v in default ${VARIANTS:-apE apT512 apE_T512 apE_T64_512}; do
  lib=""; [ $v != default ] && lib=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_$v.so
  for cfg in "4096 32" "8192 64"; do
    set -- $cfg
    SVDJ_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$1 -o run --output-format csv \
      -- python3 $R/tools/evd_ab.py --n $1 --block $2 > $O/${v}_$1.log 2>&1 || { tail -20 $O/${v}_$1.log; exit 1; }
    python3 - $O/${v}_$1 $v $1 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "apply" in r["Name"]:
            print("%-12s n=%s %-40s avg %8.1f us" % (sys.argv[2], sys.argv[3], r["Name"].split("(")[0][-40:], float(r["AverageNs"]) / 1e3))
PY
  done
  SVDJ_HIP_LIB=$lib timeout -k 10 300 python3 $R/bench.py --simulate-P 8 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
    --json-out $O/sim8_$v.json > $O/sim8_$v.log 2>&1 || { tail -20 $O/sim8_$v.log; exit 1; }
  echo "$v sim P=8: $(python3 -c "import json; print(json.load(open('$O/sim8_$v.json'))['value'])") ms/sweep"
done
