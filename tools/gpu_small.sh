# Kernel trace of the 1-GPU bench at a small size (default 4096): critical-path
# split (tools/trace_crit.py) and per-stream gaps (tools/trace_gaps.py).
# Usage (via gpurun): bash tools/gpu_small.sh [N]
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
N=${1:-4096}
O=$R/gpurun_out/small$N
mkdir -p $O
timeout -k 10 120 python3 bench.py --n $N --steps 5 --warmup 2 --no-verify > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd csv -d $O/tr -o run -- python3 $R/bench.py \
  --n $N --steps 2 --warmup 1 --no-verify > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 $R/tools/trace_crit.py $(find $O/tr -name "*.db" | head -1) | tee $O/crit.txt
python3 $R/tools/trace_gaps.py $(find $O/tr -name "*kernel_trace.csv" | head -1) | tee $O/gaps.txt | head -40
find $O/tr -name "*.db" -delete
