# Round-6 step I (dev aid): EVD micro new vs base, solve A/B at 4096^2 and 16384^2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export SVDJ_NO_AUTOBUILD=1
cd $R
for P in 8 128; do
  timeout -k 10 60 ./tools/micro/evd_bench $P 1 200 | sed 's/^/new  /' || exit 1
  timeout -k 10 60 ./tools/ab/evd_bench_base $P 1 200 | sed 's/^/base /' || exit 1
done
N=4096 timeout -k 10 600 bash tools/gpu_ab_bench.sh i4 2 || exit 1
timeout -k 10 900 bash tools/gpu_ab_bench.sh i16 2 || exit 1
