# rocprofv3 kernel stats of the two-level probe (3 sweeps of 16384^2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tlprof -o run --output-format csv -- python $R/tools/twolevel_probe.py --sizes 16384 --Wb ${1:-512} --max-sweeps 3 > $R/gpurun_out/tlprof.log 2>&1 || { tail -20 $R/gpurun_out/tlprof.log; exit 1; }
for f in $(find $R/gpurun_out/tlprof -name '*kernel_stats.csv'); do cut -d, -f1-4 $f | head -25; done
