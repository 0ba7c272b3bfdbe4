set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/twolevel_probe.py --sizes 4096,8192 --Wb 512 --verify --reps 2 > gpurun_out/tl1.log 2>&1 || { tail -30 gpurun_out/tl1.log; exit 1; }
grep '^{' gpurun_out/tl1.log
timeout -k 10 300 python -u tools/twolevel_probe.py --sizes 16384 --Wb 512 --reps 2 > gpurun_out/tl2.log 2>&1 || { tail -30 gpurun_out/tl2.log; exit 1; }
grep '^{' gpurun_out/tl2.log
timeout -k 10 300 python -u tools/twolevel_probe.py --sizes 16384 --Wb 256 --reps 2 > gpurun_out/tl3.log 2>&1 || { tail -30 gpurun_out/tl3.log; exit 1; }
grep '^{' gpurun_out/tl3.log
timeout -k 10 300 python bench.py --n 16384 --steps 1 --warmup 1 > gpurun_out/bench_16384.log 2>&1 || { tail -20 gpurun_out/bench_16384.log; exit 1; }
tail -1 gpurun_out/bench_16384.log | cut -c1-300
