#!/bin/bash
# One SOLO rank of a world-W strip job at N = 16385 (per-rank compute, no messages):
# strip_probe timings for W = 1, 2, 4, 8 and the kernel timeline of rank W/2 at W = 8.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/stl}
timeout -k 10 300 python3 scripts/strip_probe.py --n 16385 > ${OUT}_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}8 -o run -- python3 scripts/cycle_timeline.py --child --n 16385 --world 8 --rank 4 > ${OUT}.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse ${OUT}8 > ${OUT}8.json
cat ${OUT}_probe.jsonl
