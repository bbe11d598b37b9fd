#!/bin/bash
# r03 session: post checks of in-stream levels decided in their pass (k_post_dual):
# speculation tests, trace, interleaved A/B against the previous build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
D=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec_fire.py tests/test_gpu_spec.py tests/test_gpu_cross.py tests/test_gpu_strips_cross.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dual_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dual_tests.log; [ $rc -eq 0 ] || exit $rc
PGMG_LIB=$D/libpgmg_ab.so timeout -k 10 300 python3 scripts/spec_fire_trace.py 4097 40 > gpurun_out/dual_trace_4097.log 2>&1 || exit $?
grep -E "spec plan|speculates|V/s" gpurun_out/dual_trace_4097.log | tail -30
timeout -k 10 900 python3 scripts/ab_env.py --rounds 3 --grids V4097 --steps 40 \
  "base:PGMG_LIB=$D/libpgmg_base.so" "new:PGMG_LIB=$D/libpgmg.so" > gpurun_out/dual_ab_4097.jsonl 2>&1 || { tail -5 gpurun_out/dual_ab_4097.jsonl; exit 1; }
cat gpurun_out/dual_ab_4097.jsonl
timeout -k 10 900 python3 scripts/ab_env.py --rounds 3 --grids V16385,V2049 --steps 20 \
  "base:PGMG_LIB=$D/libpgmg_base.so" "new:PGMG_LIB=$D/libpgmg.so" > gpurun_out/dual_ab_16385.jsonl 2>&1 || { tail -5 gpurun_out/dual_ab_16385.jsonl; exit 1; }
cat gpurun_out/dual_ab_16385.jsonl
