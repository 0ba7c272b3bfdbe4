set -o pipefail
export SVDJ_NO_AUTOBUILD=1
echo "== acc2"; SVDJ_HIP_LIB=$GRAFT_REPO_ROOT/svd-jacobi-mpi-cuda_amd/lib/variants/libsvdj_hip_acc2.so timeout -k 10 250 python tools/probe_apply.py
