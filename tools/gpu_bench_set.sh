# Named sets of bench.py runs on one GPU (replaces the single-use round-3 scripts
# gpu_r3_final.sh / gpu_r3_configs.sh / gpu_r3_big.sh; the multi-rank rehearsal is
# tools/gpu_rehearse.sh).  Every run has its own time limit, writes its log and its
# JSON line under gpurun_out/OUT/, prints one summary line, and the first failure ends
# the script.  --progress runs print a line per sweep, so long runs are not silent.
# Usage: bash tools/gpu_bench_set.sh OUT SET [SET ...]
#   headline  16384^2 fp32, 3 timed solves
#   sigma     4096^2 / 8192^2 / 16384^2 fp32 with the fp64 sigma oracle (--check-sigma)
#   configs   tall 32768x8192 fp32 and bf16, 10000^2 fp64
#   fp64ref   the reference's fp64 job sizes: 5000^2, 20000^2, 30000^2 (accuracy block on)
#   big       65536^2 fp32 (BASELINE config 5), one solve, memory-lean accuracy check
#   sims      16384^2 rank-plan simulations P = 1, 2, 4, 8 (+ modelled links at P = 8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-benchset}; shift
mkdir -p $OUT
# verification (fp64 sigma oracle, chunked residual) runs silent after the timed
# solve: a heartbeat file under gpurun_out/ shows the call is alive meanwhile
( while true; do date >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
b() {  # tag, time limit, bench args
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u $R/bench.py "$@" > $OUT/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  tail -1 $OUT/$tag.log > $OUT/$tag.json
  python3 - $OUT/$tag.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
a = d.get("accuracy") or {}
print(sys.argv[2], "ms", d["ms_per_step"], "sweeps", d.get("sweeps"), "value", d["value"],
      "res", a.get("residual_rel"), "orth_u_max", a.get("orth_u_max_abs"),
      "sigma", a.get("sigma_max_rel_err_vs_fp64_oracle"), flush=True)
PY
}
for set in "$@"; do
  case $set in
    headline) b headline16384 400 --steps 3 --warmup 1 ;;
    sigma)
      b sigma4096 200 --n 4096 --steps 3 --warmup 1 --check-sigma
      b sigma8192 300 --n 8192 --steps 2 --warmup 1 --check-sigma
      b sigma16384 600 --n 16384 --steps 1 --warmup 0 --check-sigma --progress ;;
    configs)
      b tall_fp32 300 --m 32768 --n 8192 --steps 3 --warmup 1
      b tall_bf16 300 --m 32768 --n 8192 --dtype bf16 --steps 3 --warmup 1
      b f64_10000 300 --n 10000 --dtype fp64 --steps 2 --warmup 1 ;;
    fp64ref)
      b f64_5000 200 --n 5000 --dtype fp64 --steps 3 --warmup 1
      b f64_20000 600 --n 20000 --dtype fp64 --steps 1 --warmup 0 --progress
      b f64_30000 1000 --n 30000 --dtype fp64 --steps 1 --warmup 0 --progress ;;
    big) b big65536 1100 --n 65536 --steps 1 --warmup 0 --progress ;;
    sims)
      for P in 8 4 2 1; do b sim$P 300 --simulate-P $P --n 16384 --sim-sweeps 3; done
      b sim8_g100 300 --simulate-P 8 --n 16384 --sim-sweeps 3 --sim-link-gbps 100
      b sim8_g50 300 --simulate-P 8 --n 16384 --sim-sweeps 3 --sim-link-gbps 50 ;;
    *) echo "unknown set $set"; exit 2 ;;
  esac
done
