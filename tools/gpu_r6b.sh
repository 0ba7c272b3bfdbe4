# Round 6 measurement set (dev aid): 4096^2 and the 8-GPU rank plan under a
# kernel trace, and the default headline bench.  Logs under gpurun_out/r6b/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6b
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p4096 -o run --output-format csv -- \
  python3 $R/bench.py --n 4096 --steps 3 --warmup 1 > $O/b4096.log 2>&1 || { tail -20 $O/b4096.log; exit 1; }
tail -1 $O/b4096.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sim8 -o run --output-format csv -- \
  python3 $R/bench.py --simulate-P 8 --n 16384 --sim-sweeps 2 > $O/sim8.log 2>&1 || { tail -20 $O/sim8.log; exit 1; }
tail -1 $O/sim8.log | cut -c1-300
timeout -k 10 400 python3 $R/bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
