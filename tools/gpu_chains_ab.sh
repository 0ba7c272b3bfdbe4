set -o pipefail
export SVDJ_NO_AUTOBUILD=1
R=$GRAFT_REPO_ROOT
for n in 4096 8192; do for c in 1 2; do
timeout -k 10 300 python bench.py --n $n --steps 2 --warmup 1 --block 32 --chains $c > gpurun_out/bench_${n}_c$c.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bench_${n}_c$c.log').read().strip().splitlines()[-1]); print('n=$n chains=$c', d['value'], d['ms_per_step'], d['sweeps'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof15 -o run --output-format csv -- python $R/bench.py --n 4096 --steps 1 --warmup 1 --block 32 --chains 2 > $R/gpurun_out/prof15.log 2>&1
