# Isolated (single-stream) per-kernel times of one block sweep (dev aid).
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-16384}
cd /tmp && export TMPDIR=/tmp
run() {  # tag, W, mma, [lib]
  local tag=$1 W=$2 mma=$3
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/iso_$tag -o run --output-format csv \
    -- python $R/tools/bench_kernels.py --n $N --block $W --inner 1 --reps 1 --mma $mma \
    > $R/gpurun_out/iso_$tag.log 2>&1 || { tail -20 $R/gpurun_out/iso_$tag.log; return 1; }
  grep '^{' $R/gpurun_out/iso_$tag.log
  python - $R/gpurun_out/iso_$tag/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print("  %-48s %6s %8.1f us" % (x['Name'][:48], x['Calls'], float(x['AverageNs'])/1e3))
PY
}
run w64_nat 64 native && run w32_nat 32 native
