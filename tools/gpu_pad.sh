# Quad-step padding of ragged column counts (round 6): GPU tests of the
# touched paths, then bench.py on ragged shapes with the padding on (default)
# and off (SVDJ_DEBUG=quad_pad=0).  Usage: bash tools/gpu_pad.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pad
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_quad.py tests/test_gpu_drivers.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for shape in "4500 4097" "16400 16400"; do
  set -- $shape
  for v in on off; do
    if [ $v = off ]; then export SVDJ_DEBUG=quad_pad=0; else unset SVDJ_DEBUG; fi
    steps=3; [ $2 -gt 10000 ] && steps=1
    timeout -k 10 300 python3 -u $R/bench.py --m $1 --n $2 --steps $steps --warmup 1 \
      > $O/bench_${2}_$v.log 2>&1 || { tail -20 $O/bench_${2}_$v.log; exit 1; }
    tail -1 $O/bench_${2}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', '$v', d['ms_per_step'], d['sweeps'], d['config'].get('quad_steps'), d.get('accuracy',{}).get('residual_rel'))"
  done
done
