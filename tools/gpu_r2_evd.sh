#!/bin/bash
# GPU check after an EVD change: kernel/driver tests, 1-GPU bench at 4096 and
# 16384, the 8-GPU per-rank simulation, and per-kernel times at 4096.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  --ignore=tests/test_gpu_multirank.py > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for N in 4096 16384; do
  timeout -k 10 300 python -u bench.py --n $N --steps 2 --warmup 1 --json-out gpurun_out/bench_$N.json \
    > gpurun_out/bench_$N.log 2>&1 || { tail -20 gpurun_out/bench_$N.log; exit 1; }
  tail -1 gpurun_out/bench_$N.log
done
for P in 8 1; do
  timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 \
    --sim-sweeps 2 --json-out gpurun_out/sim_p$P.json > gpurun_out/sim_p$P.log 2>&1 \
    || { tail -30 gpurun_out/sim_p$P.log; exit 1; }
  tail -1 gpurun_out/sim_p$P.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_4096 -o run \
  --output-format csv -- python $R/bench.py --n 4096 --steps 1 --warmup 0 \
  > $R/gpurun_out/prof_4096.log 2>&1 || { tail -20 $R/gpurun_out/prof_4096.log; exit 1; }
for f in $(find $R/gpurun_out/prof_4096 -name '*kernel_stats.csv'); do cut -d, -f1-4 $f | head -12; done
