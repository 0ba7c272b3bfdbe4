# Round-6 step J (dev aid): flattened quad-apply tile distribution: quad GPU
# tests, solve A/B at 16384^2 and 4096^2, the P = 2 and P = 4 rank plans.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6j
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_quad.py -x -v --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 bash tools/gpu_ab_bench.sh j16 2 || exit 1
N=4096 timeout -k 10 600 bash tools/gpu_ab_bench.sh j4 2 || exit 1
for P in 2 4; do N=16384 P=$P bash tools/gpu_ab_sim.sh j$P 1 - || exit 1; done
