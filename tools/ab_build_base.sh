# Build tools/ab/libsvdj_hip_base.so from a git revision's block.hip (default HEAD)
# linked with the in-tree objects of the other HIP sources (A/B runs, SVDJ_HIP_LIB).
set -e
REV=${1:-HEAD}
PK=svd-jacobi-mpi-cuda_amd
T=$(mktemp -d)
git show $REV:$PK/csrc/hip/block.hip > $T/block.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$PK/csrc/include -I$PK/csrc/hip \
  -c $T/block.hip -o $T/block.o 2>/dev/null
mkdir -p tools/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/block.o \
  $(ls $PK/lib/obj/*.o | grep -v '/block.o$') -o tools/ab/libsvdj_hip_base.so
rm -rf $T
echo "built tools/ab/libsvdj_hip_base.so from $REV"
