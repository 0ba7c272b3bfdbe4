# Hardware-counter passes (rocprofv3 --pmc) over one bench solve (dev aid).
# One pass per counter group (gfx950 slots: 8 SQ, 4 TCC, 2 GRBM per pass), each
# its own run under a hard KILL timeout; a failing pass ends the script.
# Usage: bash tools/gpu_pmc.sh OUTDIR N [extra bench args]
#   PMC_CMD="python3 tools/evd_ab.py --n 4096" overrides the profiled program
#   PMC_PASSES="1 2" selects passes (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc}; N=${2:-4096}; shift 2; EXTRA="$@"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU"
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "GRBM_GUI_ACTIVE FETCH_SIZE"
  "GRBM_GUI_ACTIVE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "counter listing failed"; exit 1; }
i=0
for want in "${PASSES[@]}"; do
  i=$((i+1))
  ctr=""
  for c in $want; do  # keep the counters this box lists (a _sum suffix is derived)
    if grep -qw -- "${c%_sum}" $OUT/avail.txt; then ctr="$ctr $c"; else echo "skip $c"; fi
  done
  if [ -n "$PMC_PASSES" ] && ! [[ " $PMC_PASSES " == *" $i "* ]]; then continue; fi
  CMD=${PMC_CMD:-python3 $R/bench.py --n $N --steps 1 --warmup 0 --no-verify $EXTRA}
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d $OUT/p$i -o run --output-format csv -- \
    $CMD > $OUT/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $ctr"
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.md
# raw per-dispatch CSVs are large (> gpurun's 64 MiB merge cap): keep them compressed
tar czf $OUT/raw.tgz -C $OUT $(cd $OUT && ls -d p[0-9]*/) && rm -rf $OUT/p[0-9]*/
