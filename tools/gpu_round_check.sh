# GPU check used during development: gpu tests, default bench, kernel profile.
# Usage (from the repo root, via gpurun):  bash tools/gpu_round_check.sh [N]
set -o pipefail
# Same environment as the driver: no SVDJ_* overrides (autobuild on; in-tree libs are
# current) and pytest.ini's per-test timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-16384}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout-method thread --durations=20 \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -25 gpurun_out/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --n $N --steps 1 --warmup 1 > gpurun_out/bench_$N.log 2>&1 \
  || { tail -20 gpurun_out/bench_$N.log; exit 1; }
tail -1 gpurun_out/bench_$N.log
timeout -k 10 200 python bench.py --m 32768 --n 8192 --steps 2 --warmup 1 > gpurun_out/bench_tall.log 2>&1 \
  || { tail -20 gpurun_out/bench_tall.log; exit 1; }
tail -1 gpurun_out/bench_tall.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$N -o run \
  --output-format csv -- python $R/bench.py --n $N --steps 1 --warmup 0 \
  > $R/gpurun_out/prof_$N.log 2>&1 || { tail -20 $R/gpurun_out/prof_$N.log; exit 1; }
for f in $(find $R/gpurun_out/prof_$N -name '*kernel_stats.csv'); do cut -d, -f1-4 $f | sed -n 1,8p; done
