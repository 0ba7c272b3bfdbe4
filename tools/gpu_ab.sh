# A/B of block-path variants on one GPU (dev aid): tests, then quick_perf per mode.
set -o pipefail
export SVDJ_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?; [ $rc -le 1 ] || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }; grep -E "^FAILED|Error" gpurun_out/pytest_gpu.log | head -20
tail -2 gpurun_out/pytest_gpu.log
for mma in native bf16x6; do
  timeout -k 10 300 python tools/quick_perf.py --sizes 4096,8192 --mma $mma --verify \
    > gpurun_out/qp_$mma.log 2>&1 || { tail -20 gpurun_out/qp_$mma.log; exit 1; }
  cat gpurun_out/qp_$mma.log | cut -c1-400
done
timeout -k 10 300 python bench.py --steps 1 --warmup 1 > gpurun_out/bench_16384.log 2>&1 \
  || { tail -20 gpurun_out/bench_16384.log; exit 1; }
tail -1 gpurun_out/bench_16384.log
