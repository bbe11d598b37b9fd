#!/bin/bash
# r03 session: predicted-to-fire levels in long calls: trace, parity, long-run A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$AB timeout -k 10 300 python3 scripts/spec_fire_trace.py 2049 200 > gpurun_out/fire_trace_2049.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fire_trace_2049.log | grep -c "spec plan"; tail -3 gpurun_out/fire_trace_2049.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec_fire.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fire_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fire_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/sessions/r03_g.sh
