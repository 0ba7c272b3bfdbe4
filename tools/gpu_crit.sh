# Critical-path split (wide kernels / EVD-only / idle, tools/trace_crit.py) and
# MFMA-busy counters of simulated rank plans of 16384^2 fp32 on one GPU.
# Usage (via gpurun): bash tools/gpu_crit.sh "8 4 2 1"
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/crit
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in ${1:-8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$P -o run -- python3 $R/bench.py --simulate-P $P \
    --n ${N:-16384} --sim-sweeps 2 > $O/p$P.log 2>&1 || { tail -20 $O/p$P.log; exit 1; }
  tail -1 $O/p$P.log | cut -c1-160
  python3 $R/tools/trace_crit.py $(find $O/p$P -name "*.db" | head -1) | tee $O/p$P.crit
  find $O/p$P -name "*.db" -delete
done
# MFMA busy and wait split per kernel of the 8-GPU rank plan (one counter pass)
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmc8/p1 -o run \
  --output-format csv -- python3 $R/bench.py --simulate-P 8 --n ${N:-16384} --sim-sweeps 2 \
  > $O/pmc8.log 2>&1 || { tail -20 $O/pmc8.log; exit 1; }
python3 $R/tools/pmc_summary.py $O/pmc8 > $O/pmc8_summary.md && head -8 $O/pmc8_summary.md
