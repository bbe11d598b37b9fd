#!/bin/bash
# r03 session: tail_top129 parity (new tests + the W/V/F suites), A/B against the bulk 129
# passes (measurement build), the W-cycle timeline at 4097.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail129.py tests/test_gpu_wtail.py tests/test_gpu_parity.py tests/test_gpu_fcycle.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t129_tests.log 2>&1
rc=$?; tail -15 gpurun_out/t129_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --grids V16385,V4097,W4097,V1025 "t129:" "bulk129:AB_FLAGS=16384" > gpurun_out/t129_ab.jsonl 2>&1 || exit $?
cat gpurun_out/t129_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlW -o run -- python3 scripts/cycle_timeline.py --child --n 4097 --kind W --cycles 2 > gpurun_out/tlW.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse gpurun_out/tlW --cycles 2 > gpurun_out/tlW_4097.json || exit $?
head -c 3000 gpurun_out/tlW_4097.json
echo done
