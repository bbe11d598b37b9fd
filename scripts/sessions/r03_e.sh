#!/bin/bash
# r03 session: W(65) stage counters at 4097 (measurement build) and the W-cycle timeline
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$AB timeout -k 10 300 python3 scripts/tail_prof.py 4097 > gpurun_out/tail_prof.jsonl 2>&1 || exit $?
cat gpurun_out/tail_prof.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlW -o run -- python3 scripts/cycle_timeline.py --child --n 4097 --kind W --cycles 2 > gpurun_out/tlW.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse gpurun_out/tlW --cycles 2 > gpurun_out/tlW_4097.json || exit $?
head -c 1200 gpurun_out/tlW_4097.json
