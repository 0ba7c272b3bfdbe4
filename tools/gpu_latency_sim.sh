# One-GPU stand-in for the per-GPU shape of a P-GPU run (dev aid): n/P
# resident columns of m rows, kernel trace, per-stream gaps.
# Usage: bash tools/gpu_latency_sim.sh NLOC M [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NL=${1:-2048}; M=${2:-16384}; shift 2; EXTRA="$@"
TAG=lat_${NL}_${M}${TAGX:-}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG -o run \
  --output-format csv -- python $R/bench.py --n $NL --m $M --precondition none --steps 1 \
  --warmup 0 --no-verify $EXTRA > $R/gpurun_out/$TAG.log 2>&1 \
  || { tail -20 $R/gpurun_out/$TAG.log; exit 1; }
tail -1 $R/gpurun_out/$TAG.log | cut -c1-400
python $R/tools/trace_gaps.py $R/gpurun_out/$TAG/run_kernel_trace.csv
