# Final measurements of a round (dev aid): default bench, a kernel profile
# of one 16384^2 solve, 4096^2, svd() API timing and the rank plans.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final6
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --n 4096 --steps 10 --warmup 2 > $O/bench_4096.log 2>&1 || { tail -20 $O/bench_4096.log; exit 1; }
tail -1 $O/bench_4096.log | cut -c1-200
timeout -k 10 300 python3 -u tools/svd_api_time.py --n 16384 --reps 2 --engines pipeline > $O/svd_api.jsonl 2>&1 || { tail -20 $O/svd_api.jsonl; exit 1; }
cat $O/svd_api.jsonl
for P in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --n 16384 --simulate-P $P > $O/plan_P$P.log 2>&1 || { tail -20 $O/plan_P$P.log; exit 1; }
  tail -1 $O/plan_P$P.log | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof16384 -o run --output-format csv -- \
  python3 -u $R/bench.py --steps 1 --warmup 0 --no-verify > $O/prof16384.log 2>&1 || { tail -20 $O/prof16384.log; exit 1; }
python3 - $O/prof16384/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print("  %-50s %6s %9.1f ms %8.1f us" % (x['Name'][:50], x['Calls'], float(x['TotalDurationNs'])/1e6, float(x['AverageNs'])/1e3))
PY
