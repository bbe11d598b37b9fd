#!/bin/bash
# r03 session: the 9x9 / 5x5 tail levels in registers (lane moves, no LDS inside a visit):
# full GPU suite, tail stage clocks, interleaved A/B against the previous build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
D=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w9r_tests.log 2>&1
rc=$?; tail -4 gpurun_out/w9r_tests.log; [ $rc -eq 0 ] || exit $rc
PGMG_LIB=$D/libpgmg_ab.so timeout -k 10 300 python3 scripts/tail_prof.py 4097 > gpurun_out/tail_prof_w9r.jsonl 2>&1 || exit $?
cat gpurun_out/tail_prof_w9r.jsonl
timeout -k 10 900 python3 scripts/ab_env.py --rounds 3 --grids W4097,V4097,V16385 --steps 30 \
  "base:PGMG_LIB=$D/libpgmg_base.so" "new:PGMG_LIB=$D/libpgmg.so" > gpurun_out/w9r_ab.jsonl 2>&1 || { tail -5 gpurun_out/w9r_ab.jsonl; exit 1; }
cat gpurun_out/w9r_ab.jsonl
