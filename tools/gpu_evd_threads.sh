# EVD variants, isolated kernel times (dev aid).
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
run() {  # tag lib W
  SVDJ_HIP_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/evdt_$1 -o run --output-format csv \
    -- python $R/tools/bench_kernels.py --n 8192 --block $3 --inner 1 --reps 1 > $R/gpurun_out/evdt_$1.log 2>&1 || { tail -5 $R/gpurun_out/evdt_$1.log; return 1; }
  python - $R/gpurun_out/evdt_$1/run_kernel_stats.csv $1 <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'evd' in x['Name']: print(sys.argv[2], x['Name'][:40], x['Calls'], "%.1f us" % (float(x['AverageNs'])/1e3))
PY
}
L=$R/svd-jacobi-mpi-cuda_amd/lib
run w32 $L/libsvdj_hip.so 32 && run w64 $L/libsvdj_hip.so 64
