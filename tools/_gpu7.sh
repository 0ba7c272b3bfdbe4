set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/bench_kernels.py --n 4096 --block 32 --inner 0,1,2 > gpurun_out/bk.log 2>&1
timeout -k 10 200 python tools/bench_kernels.py --n 4096 --block 64 --inner 0,1,2 >> gpurun_out/bk.log 2>&1
timeout -k 10 200 python tools/bench_kernels.py --n 2048 --block 32 --dtype fp64 --inner 0,1,2 >> gpurun_out/bk.log 2>&1
timeout -k 10 300 python tools/quick_perf.py --sizes 2048,4096,4096 --block 32 --verify > gpurun_out/perf_w32.log 2>&1
timeout -k 10 300 python tools/quick_perf.py --sizes 4096 --block 64 --verify > gpurun_out/perf_w64.log 2>&1
cat gpurun_out/bk.log; for f in gpurun_out/perf_*.log; do grep -v amdgpu.ids $f | cut -c1-130; done
