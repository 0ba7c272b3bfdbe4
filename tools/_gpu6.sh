set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for i in 0 1 2; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof6_$i -o run --output-format csv -- python $R/tools/bench_kernels.py --n 4096 --block 32 --inner $i --reps 1 > $R/gpurun_out/prof6_$i.log 2>&1 || exit 1
done
for i in 0 1 2; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof6d_$i -o run --output-format csv -- python $R/tools/bench_kernels.py --n 2048 --block 32 --dtype fp64 --inner $i --reps 1 > $R/gpurun_out/prof6d_$i.log 2>&1 || exit 1
done
