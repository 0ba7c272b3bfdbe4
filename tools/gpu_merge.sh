# Round-6 merge-rule check (dev aid): headline bench (default), 8192^2 and
# 4096^2, then the full GPU suite and smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/merge
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
for n in 8192 4096; do
  timeout -k 10 300 python3 -u bench.py --n $n --steps 5 --warmup 1 > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], d['sweeps'], d['config']['merged_chains'], d['accuracy']['residual_rel'])"
done
bash tools/gpu_full.sh
