#!/bin/bash
# GPU session: parity of the LDS-staged coarse passes, then interleaved A/B against the
# unstaged passes (measurement build) and the rocprof timeline of the default build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_spec.py tests/test_gpu_robust_rhs.py tests/test_gpu_strips.py tests/test_gpu_fp32.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lds_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lds_tests.log; [ $rc -eq 0 ] || exit $rc
PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --grids V16385,V4097,W4097 "lds:" "nolds:PGMG_LDS_MIN_N=1000000" "lds513:PGMG_LDS_MIN_N=513" > gpurun_out/lds_ab.jsonl 2>&1 || exit $?
cat gpurun_out/lds_ab.jsonl
bash scripts/timeline.sh gpurun_out/tl_lds > /dev/null 2>&1 || exit $?
