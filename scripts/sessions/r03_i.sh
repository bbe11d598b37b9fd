#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$AB timeout -k 10 300 python3 scripts/spec_fire_trace.py 2049 40 > gpurun_out/fire_trace_2049_40.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fire_trace_2049_40.log
