#!/bin/bash
# Kernel trace of the bench's call shape at N = 4097 (3 + 10 cycles), the raw CSV kept: where
# the device idles between launches (host-bound stretches, validation round trips).
set -u
export TMPDIR=/tmp
OUT=${1:-gpurun_out/gap}
mkdir -p ${OUT}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/raw -o run -- python3 scripts/cycle_timeline.py --child --n ${2:-4097} --cycles 10 --flags ${3:-0} > ${OUT}/child.log 2>&1 || exit $?
f=$(find ${OUT}/raw -name '*kernel_trace.csv' | head -1)
cp "$f" ${OUT}/kernel_trace.csv
rm -rf ${OUT}/raw
