#!/bin/bash
# Host AddressSanitizer + UBSan run of the CPU test suite against instrumented
# builds of libsvdj_cpu.so (schedules, CPU oracle, reference input generator,
# verification, stop rule) and of libsvdj_dist.so's host code (id-file
# handshake, plan / pair-list builder, watchdog).  GPU sanitizers are not
# available on this pool; the kernels are not covered.
# Usage: bash tools/asan_cpu_tests.sh [pytest args]
set -o pipefail
cd "$(dirname "$0")/.."
read -r CPU DIST < <(python3 -c "
import importlib; b = importlib.import_module('svd-jacobi-mpi-cuda_amd._build')
print(b.build_cpu(asan=True), b.build_dist_asan())") || exit 1
export SVDJ_CPU_LIB=$CPU SVDJ_DIST_LIB=$DIST
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
# the whole CPU suite unless test paths are given
WHAT=tests
for a in "$@"; do case "$a" in tests/*) WHAT= ;; esac; done
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  python3 -m pytest $WHAT -q -m "not gpu" -p no:cacheprovider "$@"
