# The reference's own run shape (build/runSVDMPICUDAWithoutCMake.slurm:30-33:
# mpiexec -n 2, fp64, n = 5000 .. 30000), on the one-GPU box:
#   * root-owned A on rank 0, 2 ranks sharing the GPU over RCCL (socket
#     transport -- the ranks time-share one device, so these times are NOT a
#     2-GPU speedup), scatter + sweeps + gather of U, S, V timed like the
#     reference (main.cu:1586-1611), verified after the timed region;
#   * the native launcher (svdj_dist_main --np 2 --verify: fp64 host check);
#   * rank 0's P=2 plan simulated at 20000 / 30000 (per-sweep time).
# Usage (from the repo root, via gpurun): bash tools/gpu_refshape.sh
set -o pipefail
O=gpurun_out/refshape
mkdir -p $O
export SVDJ_SHARED_GPU=1
for n in 5000 10000; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + n / 1000)) bench.py --gpus 2 --size $n \
    --dtype fp64 --root-owned --steps 1 --warmup 1 --json-out $O/root_p2_fp64_$n.json \
    > $O/root_p2_fp64_$n.log 2>&1 || { tail -20 $O/root_p2_fp64_$n.log; exit 1; }
  tail -1 $O/root_p2_fp64_$n.log | cut -c1-160
done
timeout -k 10 300 svd-jacobi-mpi-cuda_amd/bin/svdj_dist_main 5000 --np 2 --shared-gpu --dtype f64 \
  --verify --warmup 1 --timeout 250 > $O/native_p2_fp64_5000_triu.log 2>&1 \
  || { tail -20 $O/native_p2_fp64_5000_triu.log; exit 1; }
grep -E "time|sweeps|USVt|TU|TV" $O/native_p2_fp64_5000_triu.log
for n in 20000 30000; do
  timeout -k 10 400 python bench.py --simulate-P 2 --n $n --dtype fp64 --sim-sweeps 2 \
    --json-out $O/sim_p2_fp64_$n.json > $O/sim_p2_fp64_$n.log 2>&1 \
    || { tail -20 $O/sim_p2_fp64_$n.log; exit 1; }
  tail -1 $O/sim_p2_fp64_$n.log | cut -c1-140
done
