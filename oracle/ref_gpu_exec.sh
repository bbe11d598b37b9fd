#!/bin/bash
# oracle/ref_gpu_exec.sh OUT — the reference's own gpu_exec entry (3_part_parallel/main.cu)
# built against this repository's C++ mirror and libpgmg.so, with exactly the two edits
# INTEGRATION.md §2 documents (TEST INFRASTRUCTURE: the check that the reference-side
# switch-over compiles and runs):
#   1. #include "ParallelTestRunner.cu"  ->  #include "ParallelTestRunner.hpp" (host/)
#   2. the CUDA warm-up block (cudaMallocManaged / cudaDeviceSynchronize / cudaFree,
#      main.cu:8-13)  ->  pgmg_device_sync();
# The edited source is piped to g++ (no copy of it is written); the reference's CPU runner
# (2_part_MG/MultiGridTestRunner.hpp, included by main.cu) and globals.cpp are compiled
# where they lie.  Needs the reference tree (this container only); the binary travels.
set -euo pipefail
OUT=${1:?usage: ref_gpu_exec.sh OUT}
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
PKG="$HERE/../parallel-geometric-multigrid-for-poisson-problem_amd"
sed -e 's|#include "ParallelTestRunner.cu"|#include "ParallelTestRunner.hpp"|' \
    -e '/Allocate managed memory for temporary data/,/cudaFree(tmp);/c\    pgmg_device_sync();' \
    "$REF/3_part_parallel/main.cu" |
  ${CXX:-g++} -std=c++17 -O2 -ffp-contract=off -w -I"$HERE/../include" -I"$PKG/host" \
    -I"$REF/3_part_parallel" -x c++ - -x none "$REF/globals.cpp" -L"$PKG" -lpgmg \
    -Wl,-rpath,'$ORIGIN/../../parallel-geometric-multigrid-for-poisson-problem_amd' -o "$OUT"
