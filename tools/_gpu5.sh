set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/quick_perf.py --sizes 2048,4096,4096 --block 32 > gpurun_out/perf_w32.log 2>&1
SVDJ_HIP_LIB=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_evd256.so timeout -k 10 300 python tools/quick_perf.py --sizes 2048,4096,4096 --block 32 > gpurun_out/perf_w32_evd256.log 2>&1
timeout -k 10 300 python tools/quick_perf.py --sizes 4096,4096 --block 64 > gpurun_out/perf_w64.log 2>&1
SVDJ_HIP_LIB=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_evd256.so timeout -k 10 300 python tools/quick_perf.py --sizes 4096,4096 --block 64 > gpurun_out/perf_w64_evd512.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5 -o run --output-format csv -- python $R/tools/quick_perf.py --sizes 4096 --block 32 > $R/gpurun_out/prof5.log 2>&1
cd $R
tail -3 gpurun_out/gpu_tests.log; for f in gpurun_out/perf_*.log; do echo $f; grep -v amdgpu.ids $f | cut -c1-150; done
