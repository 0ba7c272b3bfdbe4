# A/B of measurement-only kernel variants (tools/kernel_ab.py) on simulated
# rank plans of 16384^2 fp32, full-work sweeps.  Replaces the box copy's
# libsvdj_hip.so per variant and restores it: run only through gpurun.
# Usage: bash tools/gpu_kernel_ab.sh "nogram fused" "1 8"
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/ab
mkdir -p $O $R/tools/micro/scratch
LIB=$R/svd-jacobi-mpi-cuda_amd/lib/libsvdj_hip.so
export SVDJ_NO_AUTOBUILD=1
cp $LIB $R/tools/micro/scratch/libsvdj_hip.base.so
run() {  # name P
  timeout -k 10 200 python3 bench.py --simulate-P $2 --n ${N:-16384} --sim-sweeps 2 > $O/$1_p$2.json \
    2> $O/$1_p$2.err || { tail $O/$1_p$2.err; exit 1; }
  echo "$1 P=$2 $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value'])" $O/$1_p$2.json) ms/sweep"
}
for P in ${2:-1}; do run base $P; done
for v in ${1:-nogram}; do
  python3 tools/kernel_ab.py $v $LIB > $O/build_$v.log 2>&1 || { tail $O/build_$v.log; exit 1; }
  for P in ${2:-1}; do run $v $P; done
done
cp $R/tools/micro/scratch/libsvdj_hip.base.so $LIB
for P in ${2:-1}; do run base_end $P; done
