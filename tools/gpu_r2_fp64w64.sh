set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_kern.log 2>&1 || { tail -40 gpurun_out/pytest_kern.log; exit 1; }
tail -1 gpurun_out/pytest_kern.log
timeout -k 10 300 python -u bench.py --n 8192 --dtype fp64 --block 64 --steps 1 --warmup 1 --json-out gpurun_out/cfg/fp64_8192_w64.json > gpurun_out/cfg/fp64_8192_w64.log 2>&1 || { tail -20 gpurun_out/cfg/fp64_8192_w64.log; exit 1; }
tail -1 gpurun_out/cfg/fp64_8192_w64.log | cut -c 1-900
timeout -k 10 300 python -u bench.py --n 8192 --dtype fp64 --block 32 --steps 1 --warmup 1 --json-out gpurun_out/cfg/fp64_8192_w32.json > gpurun_out/cfg/fp64_8192_w32.log 2>&1 || { tail -20 gpurun_out/cfg/fp64_8192_w32.log; exit 1; }
tail -1 gpurun_out/cfg/fp64_8192_w32.log | cut -c 1-900
timeout -k 10 600 python -u bench.py --n 16384 --dtype fp64 --block 64 --steps 1 --warmup 0 --no-verify --json-out gpurun_out/cfg/fp64_16384_w64.json > gpurun_out/cfg/fp64_16384_w64.log 2>&1 || { tail -20 gpurun_out/cfg/fp64_16384_w64.log; exit 1; }
tail -1 gpurun_out/cfg/fp64_16384_w64.log | cut -c 1-900
