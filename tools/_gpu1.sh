set -o pipefail
export SVDJ_NO_AUTOBUILD=1
rocminfo | grep -m3 -E "gfx950|Marketing" > gpurun_out/devinfo.txt || true
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/quick_perf.py --sizes 1024,2048,4096 --verify > gpurun_out/perf_f32.log 2>&1
timeout -k 10 200 python tools/quick_perf.py --sizes 1024,2048 --dtype fp64 --verify > gpurun_out/perf_f64.log 2>&1
timeout -k 10 200 python tools/quick_perf.py --sizes 1024 --method scalar --verify > gpurun_out/perf_scalar.log 2>&1
tail -5 gpurun_out/gpu_tests.log; cat gpurun_out/perf_*.log
