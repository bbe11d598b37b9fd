#!/bin/bash
# rocprofv3 kernel traces of one timed V-cycle call at N = 16385 and 4097, parsed into
# per-kernel busy time and inter-kernel gaps per cycle (scripts/cycle_timeline.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/tl}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}16385 -o run -- python3 scripts/cycle_timeline.py --child --n 16385 > ${OUT}.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}4097 -o run -- python3 scripts/cycle_timeline.py --child --n 4097 --cycles 40 >> ${OUT}.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse ${OUT}16385 > ${OUT}16385.json
python3 scripts/cycle_timeline.py --parse ${OUT}4097 --cycles 40 > ${OUT}4097.json
head -c 1500 ${OUT}16385.json
