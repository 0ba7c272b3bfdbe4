# Refresh the measured-performance table (dev aid): fp32 sizes on one GPU and
# the 16384^2 rank plans, current build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sizes6
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
for n in 8192 12288; do
  timeout -k 10 600 python3 -u bench.py --n $n --steps 2 --warmup 1 > $O/b$n.log 2>&1 || { tail -20 $O/b$n.log; exit 1; }
  tail -1 $O/b$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=d.get('accuracy') or {}; print($n, d['ms_per_step'], d['sweeps'], a.get('residual_rel'), a.get('orth_u_max_abs'), a.get('sigma_max_rel_err_vs_fp64_oracle'))"
done
timeout -k 10 600 python3 -u bench.py --m 32768 --n 8192 --steps 2 --warmup 1 > $O/b32768x8192.log 2>&1 || { tail -20 $O/b32768x8192.log; exit 1; }
tail -1 $O/b32768x8192.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=d.get('accuracy') or {}; print('32768x8192', d['ms_per_step'], d['sweeps'], a.get('residual_rel'), a.get('sigma_max_rel_err_vs_fp64_oracle'))"
for P in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --n 16384 --simulate-P $P > $O/plan_P$P.log 2>&1 || { tail -20 $O/plan_P$P.log; exit 1; }
  tail -1 $O/plan_P$P.log | cut -c1-150
done
