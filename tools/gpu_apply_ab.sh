# Native apply variants, isolated (dev aid).
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
run() {  # tag lib W
  SVDJ_HIP_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_$1 -o run --output-format csv \
    -- python $R/tools/bench_kernels.py --n 16384 --block $3 --inner 1 --reps 1 > $R/gpurun_out/ab_$1.log 2>&1 || { tail -5 $R/gpurun_out/ab_$1.log; return 1; }
  python - $R/gpurun_out/ab_$1/run_kernel_stats.csv $1 <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'apply' in x['Name']: print(sys.argv[2], x['Name'][:40], x['Calls'], "%.1f us" % (float(x['AverageNs'])/1e3))
PY
}
L=$R/svd-jacobi-mpi-cuda_amd/lib
run base $L/libsvdj_hip.so 64 && run t512 $L/variants/libsvdj_hip_t512.so 64 && run qpd16 $L/variants/libsvdj_hip_qpd16.so 64
