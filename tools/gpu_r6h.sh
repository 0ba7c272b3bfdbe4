# Round-6 step H (dev aid): tangent-only EVD records + decoupled rotation
# test: GPU tests, EVD micro (new, base, ablations), solve A/B at 4096^2 and
# 16384^2, the P = 8 rank plan.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6h
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_drivers.py tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for P in 8 32 128; do
  timeout -k 10 60 ./tools/micro/evd_bench $P 1 200 | sed 's/^/new  /' || exit 1
  timeout -k 10 60 ./tools/ab/evd_bench_base $P 1 200 | sed 's/^/base /' || exit 1
done
timeout -k 10 60 ./tools/micro/evd_bench_abl 8 1 200 || exit 1
N=4096 timeout -k 10 600 bash tools/gpu_ab_bench.sh h4 2 || exit 1
timeout -k 10 900 bash tools/gpu_ab_bench.sh h16 2 || exit 1
N=16384 P=8 bash tools/gpu_ab_sim.sh h8 1 - || exit 1
N=4096 STEPS=10 bash tools/gpu_ab_knobs.sh h4k 1 - "quad_gram_chunks=8" "quad_gram_chunks=4" || exit 1
