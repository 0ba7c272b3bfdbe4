#!/bin/bash
# EVD phase split (SVDJ_EVD_PROFILE variant) in the per-GPU shape of the
# 8-GPU 16384^2 job (8 pairs, 16384 rows) and the 1-GPU shape.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/evdprof
mkdir -p $O
export SVDJ_NO_AUTOBUILD=1
export SVDJ_HIP_LIB=$(pwd)/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_prof.so
timeout -k 10 120 python3 tools/evd_phase_profile.py --m 16384 --pairs 8 --cases fp32:64,fp32:32 > $O/p8.jsonl 2>&1 || { cat $O/p8.jsonl; exit 1; }
timeout -k 10 120 python3 tools/evd_phase_profile.py --m 16384 --pairs 8 --cases fp32:64 --order cyclic >> $O/p8.jsonl 2>&1 || { cat $O/p8.jsonl; exit 1; }
cat $O/p8.jsonl
