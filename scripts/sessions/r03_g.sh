#!/bin/bash
# r03 session: long runs (coarse levels converge and fire): predicted-to-fire + segment
# planning vs the r02 policy (PGMG_FLAG_NO_SPEC_FIRE), interleaved, hash-checked per run
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --steps 200 --grids V4097,V2049 "fire:" "r02:AB_FLAGS=8192" > gpurun_out/long_ab.jsonl 2>&1 || exit $?
timeout -k 10 600 python3 scripts/ab_env.py --rounds 2 --steps 100 --grids V16385 "fire:" "r02:AB_FLAGS=8192" >> gpurun_out/long_ab.jsonl 2>&1 || exit $?
cat gpurun_out/long_ab.jsonl
