#!/bin/bash
# r03 session (tail variants): W/V tail parity, then
# interleaved A/B against the previous build (libpgmg_base.so) and the stage counters
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
PKG=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_wtail.py tests/test_gpu_parity.py tests/test_gpu_fcycle.py tests/test_gpu_fp32.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --grids W4097,V4097 "r2:" "base:PGMG_LIB=$PKG/libpgmg_base.so" > gpurun_out/r2_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r2_ab.jsonl
PGMG_LIB=$PKG/libpgmg_ab.so timeout -k 10 300 python3 scripts/tail_prof.py 4097 > gpurun_out/tail_prof_r2.jsonl 2>&1 || exit $?
cat gpurun_out/tail_prof_r2.jsonl
