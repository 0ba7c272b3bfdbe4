# Round-6 step C (dev aid): quad-step GPU tests on the in-tree build, the
# quad Gram micro-ablations, then an interleaved solve A/B against the base build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6c
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -x -v --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 ./tools/micro/quad_apply_ab > $O/micro.jsonl 2> $O/micro.err || { tail -5 $O/micro.err; exit 1; }
grep gram_quad $O/micro.jsonl
timeout -k 10 900 bash tools/gpu_ab_bench.sh gram16 ${REPS:-2}
