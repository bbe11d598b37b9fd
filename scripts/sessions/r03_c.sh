#!/bin/bash
# r03 session: levels predicted to fire + segment planning: parity (new tests, the speculation
# and full-size suites), interleaved A/B against PGMG_FLAG_NO_SPEC_FIRE (the r02 policy) at
# the bench's call shapes, the 4097 timeline of a 3 + 40 call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec_fire.py tests/test_gpu_spec.py tests/test_gpu_fullsize.py tests/test_gpu_dropin.py tests/test_gpu_robust_rhs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fire_tests.log 2>&1
rc=$?; tail -15 gpurun_out/fire_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --steps 40 --grids V4097,V2049 "fire:" "r02:AB_FLAGS=8192" > gpurun_out/fire_ab.jsonl 2>&1 || exit $?
cat gpurun_out/fire_ab.jsonl
timeout -k 10 600 python3 scripts/ab_env.py --rounds 2 --steps 20 --grids V16385 "fire:" "r02:AB_FLAGS=8192" >> gpurun_out/fire_ab.jsonl 2>&1 || exit $?
tail -2 gpurun_out/fire_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_fire -o run -- python3 scripts/cycle_timeline.py --child --n 4097 --cycles 40 > gpurun_out/tl_fire.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse gpurun_out/tl_fire --cycles 40 > gpurun_out/tl_fire_4097.json || exit $?
head -c 1500 gpurun_out/tl_fire_4097.json
echo done
