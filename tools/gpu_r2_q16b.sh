set -o pipefail
cd /root/repo
R=$(pwd); O=gpurun_out/q16; mkdir -p $O; export SVDJ_NO_AUTOBUILD=1
for v in off on; do
  L=""; [ $v = off ] && L=$R/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_q16off.so
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --simulate-P 2 --simulate-rank 0 --n 16384 --sim-sweeps 2 \
    --json-out $O/p2_$v.json > $O/p2_$v.log 2>&1 || { tail -20 $O/p2_$v.log; exit 1; }
  echo "q16=$v P=2: $(python3 -c "import json; print(json.load(open('$O/p2_$v.json'))['value'])")"
  SVDJ_HIP_LIB=$L timeout -k 10 300 python -u bench.py --n 16384 --steps 2 --warmup 1 --json-out $O/one_$v.json > $O/one_$v.log 2>&1 || { tail -20 $O/one_$v.log; exit 1; }
  echo "q16=$v 1-GPU: $(python3 -c "import json; d=json.load(open('$O/one_$v.json')); print(d['ms_per_step'], d['sweeps'])")"
done
