# Round-6 step E (dev aid): GPU tests of the quad path and the drivers, then
# the solve A/B against the base build, 4096^2 with the new issue rules, and
# one sigma-checked 16384^2 run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6e
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_drivers.py -x -v --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 bash tools/gpu_ab_bench.sh split8 2 || exit 1
timeout -k 10 300 python3 -u bench.py --n 4096 --steps 10 --warmup 2 > $O/b4096.log 2>&1 || { tail -20 $O/b4096.log; exit 1; }
tail -1 $O/b4096.log | cut -c1-400
timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 0 --check-sigma > $O/sigma.log 2>&1 || { tail -20 $O/sigma.log; exit 1; }
tail -1 $O/sigma.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['sweeps'], d['accuracy'], d.get('sigma_check'))"
