#!/bin/bash
# EVD A/B: isolated per-kernel latency (single stream, rocprofv3 stats) for
# the default library and variants, the phase profile, then end-to-end numbers.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out/ab
export SVDJ_NO_AUTOBUILD=1
V=$R/svd-jacobi-mpi-cuda_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_kern.log 2>&1 || { tail -40 gpurun_out/pytest_kern.log; exit 1; }
tail -2 gpurun_out/pytest_kern.log
for v in prof profq32; do
  SVDJ_HIP_LIB=$V/libsvdj_hip_$v.so timeout -k 10 120 python tools/evd_phase_profile.py > gpurun_out/ab/phase_$v.log 2>&1 || { tail -20 gpurun_out/ab/phase_$v.log; exit 1; }
  echo "== phase $v"; cat gpurun_out/ab/phase_$v.log
done
cd /tmp && export TMPDIR=/tmp
run() {  # name lib n W
  local name=$1 lib=$2 n=$3 W=$4
  if [ "$lib" != default ]; then export SVDJ_HIP_LIB=$V/$lib; else unset SVDJ_HIP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/$name -o run --output-format csv \
    -- python $R/tools/evd_ab.py --n $n --block $W > $R/gpurun_out/ab/$name.log 2>&1 || { tail -20 $R/gpurun_out/ab/$name.log; exit 1; }
  grep ms_per_sweep $R/gpurun_out/ab/$name.log
  python3 - "$R/gpurun_out/ab/$name" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "svdj" in r["Name"] and ("evd" in r["Name"] or "apply" in r["Name"]):
            print("   %-40s calls %6s avg %9.1f us" % (r["Name"].split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run w32_default default 4096 32
run w32_t512 libsvdj_hip_t512.so 4096 32
run w32_q32 libsvdj_hip_q32.so 4096 32
run w64_default default 8192 64
run w64_q32 libsvdj_hip_q32.so 8192 64
unset SVDJ_HIP_LIB
cd $R
for lib in default q32; do
  for N in 8192 16384; do
    if [ "$lib" != default ]; then export SVDJ_HIP_LIB=$V/libsvdj_hip_$lib.so; else unset SVDJ_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --n $N --steps 1 --warmup 1 > gpurun_out/bench_${lib}_$N.log 2>&1 || { tail -20 gpurun_out/bench_${lib}_$N.log; exit 1; }
    echo "== bench $lib $N"; tail -1 gpurun_out/bench_${lib}_$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['sweeps'], d['accuracy'])"
  done
done
unset SVDJ_HIP_LIB
timeout -k 10 300 python -u bench.py --simulate-P 8 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
  > gpurun_out/sim_p8.log 2>&1 || { tail -30 gpurun_out/sim_p8.log; exit 1; }
tail -1 gpurun_out/sim_p8.log
