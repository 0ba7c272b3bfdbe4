set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6a
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_drivers.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/svd_api_time.py --n 16384 --reps 2 > $O/svd_api.jsonl 2>&1 || { tail -20 $O/svd_api.jsonl; exit 1; }
cat $O/svd_api.jsonl
timeout -k 10 300 bash tools/gpu_prof.sh 16384 bf16x6 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cat $O/prof.log
