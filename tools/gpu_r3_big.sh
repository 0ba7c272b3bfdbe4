# BASELINE config 5 on one GPU (65536^2 fp32, to convergence) with the default
# split-bf16 apply; --progress prints one line per sweep (dev aid).
set -o pipefail
O=gpurun_out/r3big; mkdir -p $O
timeout -k 10 1000 python3 -u bench.py --n 65536 --steps 1 --warmup 0 --no-verify --progress > $O/big65536.log 2>&1 || { tail -5 $O/big65536.log; exit 1; }
tail -1 $O/big65536.log | cut -c1-600
