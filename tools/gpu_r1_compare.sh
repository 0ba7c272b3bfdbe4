# Before/after: the round-1 library (built from git 536860a into lib/variants/libsvdj_hip_r1.so)
# timed with tools/evd_ab_r1.py, single stream, plus its EVD PMC passes.
set -o pipefail
R=$(pwd); export SVDJ_NO_AUTOBUILD=1
export SVDJ_HIP_LIB=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_r1.so
mkdir -p gpurun_out/r1
cd /tmp && export TMPDIR=/tmp
for cfg in "4096 32" "8192 64"; do set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1/n$1 -o run --output-format csv -- python $R/tools/evd_ab_r1.py --n $1 --block $2 > $R/gpurun_out/r1/n$1.log 2>&1 || { tail -20 $R/gpurun_out/r1/n$1.log; exit 1; }
  tail -1 $R/gpurun_out/r1/n$1.log
  python3 - $R/gpurun_out/r1/n$1 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "svdj" in r["Name"]:
            print("   %-40s calls %6s avg %9.1f us" % (r["Name"].split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
cd $R
PMC_PASSES="1 2" PMC_CMD="python3 $R/tools/evd_ab_r1.py --n 4096 --block 32 --sweeps 1" bash tools/gpu_pmc.sh pmc_evd32_r1 4096 > /dev/null && grep "evd_kernel" gpurun_out/pmc_evd32_r1/summary.md | head -3
