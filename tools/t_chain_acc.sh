set -o pipefail
export SVDJ_NO_AUTOBUILD=1
for c in 1 2; do
timeout -k 10 200 python bench.py --n 8192 --steps 1 --warmup 0 --mma bf16x6 --chains $c > gpurun_out/c$c.log 2>&1 || { tail gpurun_out/c$c.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/c$c.log').read().strip().splitlines()[-1]); print('chains $c', d['ms_per_step'], d['sweeps'], d['accuracy'])"
done
timeout -k 10 200 python tools/quick_perf.py --sizes 8192 --mma bf16x6 --verify | cut -c1-100
timeout -k 10 200 python tools/quick_perf.py --sizes 8192 --mma bf16x6 --verify | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:v for k,v in d.items() if k!='hist'})"
