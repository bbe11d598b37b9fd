#!/bin/bash
# rocprofv3 kernel statistics of the drop-in path (gpu_exec: 3 + 20 one-cycle
# ParallelMultiGridSolver::v_cycle calls on device arrays in place at N = 16385) beside the
# context API's one-cycle calls (bench.py's context_single_calls shape).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
EXE=parallel-geometric-multigrid-for-poisson-problem_amd/host/gpu_exec
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dropin -o run -- $EXE --n 16385 --cycles 20 --warmup 3 --v-only --hash > gpurun_out/prof_dropin.log 2>&1 || exit $?
head -12 gpurun_out/prof_dropin/*/run_kernel_stats.csv 2>/dev/null || find gpurun_out/prof_dropin -name "*stats*"
