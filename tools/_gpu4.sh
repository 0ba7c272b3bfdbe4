set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/quick_perf.py --sizes 2048,4096 --block 32 --verify > gpurun_out/perf_w32.log 2>&1
timeout -k 10 300 python tools/quick_perf.py --sizes 4096 --block 64 --verify > gpurun_out/perf_w64.log 2>&1
timeout -k 10 300 python tools/quick_perf.py --sizes 2048 --dtype fp64 --verify > gpurun_out/perf_f64.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof4 -o run --output-format csv -- python $R/tools/quick_perf.py --sizes 4096 --block 32 > $R/gpurun_out/prof4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof4b -o run --output-format csv -- python $R/tools/quick_perf.py --sizes 4096 --block 64 > $R/gpurun_out/prof4b.log 2>&1
cd $R
timeout -k 10 500 python bench.py --n 16384 --steps 1 --warmup 0 > gpurun_out/bench_16384.log 2>&1
tail -3 gpurun_out/gpu_tests.log; cat gpurun_out/perf_*.log gpurun_out/bench_16384.log | grep -v amdgpu.ids
