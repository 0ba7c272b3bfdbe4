#!/bin/bash
# LDS-staged cross Gram: kernel tests, then A/B against the register-fragment
# Gram (SVDJ_GRAM_LDS=0) on the 1-GPU headline and the 8/2-GPU rank plans.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/gramlds
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${VARIANTS:-4 3 2 0}; do
  for P in ${PS:-8 2}; do
    SVDJ_GRAM_LDS=$v timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --sim-sweeps 2 \
      --json-out $O/sim_p${P}_lds$v.json > $O/sim_p${P}_lds$v.log 2>&1 || { tail -20 $O/sim_p${P}_lds$v.log; exit 1; }
    echo "lds=$v sim P=$P: $(python3 -c "import json; print(json.load(open('$O/sim_p${P}_lds$v.json'))['value'])") ms/sweep"
  done
  SVDJ_GRAM_LDS=$v timeout -k 10 300 python -u bench.py --n 16384 --steps 1 --warmup 1 --json-out $O/one_lds$v.json \
    > $O/one_lds$v.log 2>&1 || { tail -20 $O/one_lds$v.log; exit 1; }
  echo "lds=$v 1-GPU 16384: $(python3 -c "import json; d=json.load(open('$O/one_lds$v.json')); print(d['ms_per_step'], 'ms', d['sweeps'], d['accuracy'])")"
done
