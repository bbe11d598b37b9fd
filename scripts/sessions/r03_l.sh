#!/bin/bash
# r03 session: W-cycle plans over long runs of one-cycle calls, against no plans (NO_SPEC_FIRE),
# interleaved twice
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
D=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
for r in 1 2; do
  for f in 0 8192; do
    PGMG_TRACE_FLAGS=$f timeout -k 10 300 python3 scripts/spec_fire_trace.py 4097 1 W 16 > gpurun_out/wlong_${f}_$r.log 2>&1 || exit $?
    grep -E "flags=|call 15" gpurun_out/wlong_${f}_$r.log
  done
done
for f in 0 8192; do
  PGMG_TRACE_FLAGS=$f timeout -k 10 300 python3 scripts/spec_fire_trace.py 1025 1 W 30 > gpurun_out/wlong1025_$f.log 2>&1 || exit $?
  grep -E "flags=|call 29" gpurun_out/wlong1025_$f.log
done
