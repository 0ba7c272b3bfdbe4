# Effective shader clock per quad-kernel variant of tools/micro/quad_apply_ab
# (dev aid): GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time (MI355X_MICROARCH
# "DVFS give-back"), with MFMA-busy cycles.  One counter pass + kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/clock
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES \
  -d $O/run -o run --output-format csv -- $R/tools/micro/quad_apply_ab > $O/micro.log 2>&1 \
  || { tail -20 $O/micro.log; exit 1; }
python3 $R/tools/clock_summary.py $O/run > $O/summary.txt && cat $O/summary.txt
