#!/bin/bash
# Bank-conflict-optimised EVD dealing (tools/evd_deal_opt.py) vs the round-2
# dealing (variant lib built with -DSVDJ_EVD_DEAL_OPT=0): kernel tests, rank
# plans, 1-GPU headline, and the EVD's LDS bank-conflict PMC counters.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/deal
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
OLD=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_dealold.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old; do
  L=""; [ $v = old ] && L=$OLD
  for P in 8 4 2; do
    SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --json-out $O/sim_p${P}_$v.json > $O/sim_p${P}_$v.log 2>&1 || { tail -20 $O/sim_p${P}_$v.log; exit 1; }
    echo "$v sim P=$P: $(python3 -c "import json; print(json.load(open('$O/sim_p${P}_$v.json'))['value'])") ms/sweep"
  done
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --json-out $O/one_$v.json \
    > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  echo "$v 1-GPU 16384: $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], 'ms', d['sweeps'], d['accuracy'])")"
done
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  L=""; [ $v = old ] && L=$OLD
  SVDJ_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
    --kernel-trace --stats -d $R/$O/pmc_$v -o run --output-format csv -- python $R/bench.py --simulate-P 8 --simulate-rank 0 \
    --n 16384 --sim-sweeps 1 > $R/$O/pmc_$v.log 2>&1 || { tail -20 $R/$O/pmc_$v.log; exit 1; }
  python3 - $R/$O/pmc_$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"][:40]
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in tot.items():
    if "evd" in k and v.get("SQ_LDS_IDX_ACTIVE"):
        print(sys.argv[1].split("/")[-1], k, "bank conflict share %.1f %%" % (100 * v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]),
              "LDS cycles %.3g" % v["SQ_LDS_IDX_ACTIVE"])
PY
done
