# Round-6 step G (dev aid): tests, EVD micro new vs base, solve A/B at
# 16384^2 and 4096^2, rank plans P = 4, 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6g
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_drivers.py tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for P in 8 32 128; do for nc in 1 4; do
  timeout -k 10 60 ./tools/micro/evd_bench $P $nc 200 | sed 's/^/new  /' || exit 1
  timeout -k 10 60 ./tools/ab/evd_bench_base $P $nc 200 | sed 's/^/base /' || exit 1
done; done
timeout -k 10 900 bash tools/gpu_ab_bench.sh g16 2 || exit 1
N=4096 timeout -k 10 600 bash tools/gpu_ab_bench.sh g4 2 || exit 1
N=16384 P=8 bash tools/gpu_ab_sim.sh g8 1 - || exit 1
N=16384 P=4 bash tools/gpu_ab_sim.sh g4p 1 - || exit 1
