set -o pipefail
cd /root/repo; export SVDJ_NO_AUTOBUILD=1; O=gpurun_out/f64awg; mkdir -p $O
for t in "" 2048; do
  for P in 2 4; do
    SVDJ_APPLY_WG_TARGET=$t timeout -k 10 300 python -u bench.py --simulate-P $P --simulate-rank 0 --n 16384 --dtype fp64 --sim-sweeps 1 \
      --json-out $O/p${P}_t$t.json > $O/p${P}_t$t.log 2>&1 || { tail -20 $O/p${P}_t$t.log; exit 1; }
    echo "fp64 target=${t:-rule} P=$P: $(python3 -c "import json; d=json.load(open('$O/p${P}_t$t.json')); print(d['value'], d['config']['block_W'])")"
  done
done
