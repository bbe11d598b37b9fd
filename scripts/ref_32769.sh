#!/bin/bash
# The reference's own MultigridSolver (oracle/_ref/ref_harness: the reference's headers compiled
# in place, oracle/Makefile) at N = 32769 -- ~70 GB of host memory, more than the build container
# has, so it runs on the GPU box's host (no GPU used).  Its per-cycle hashes and sweep counts
# are compared with tests/golden/cycles.json's 32769 rows, which came from the restatement
# (scripts/check_ref_32769.py).   bash scripts/ref_32769.sh OUT KIND CYCLES LIMIT
set -u
OUT=${1:-gpurun_out/ref32769}
KIND=${2:-V}
CYC=${3:-6}
LIM=${4:-1000}
mkdir -p ${OUT}
# a line a minute: the cycles of a 32769 grid on one core take longer than the idle limit
( for i in $(seq 40); do sleep 50; echo "hb ${i} $(date +%T)"; done ) &
HB=$!
timeout -k 10 ${LIM} oracle/_ref/ref_harness ${KIND} 32769 ${CYC} 1e-7 > ${OUT}/${KIND}.out 2> ${OUT}/${KIND}.err
rc=$?
kill ${HB} 2>/dev/null
echo "${KIND} rc=${rc}"
cat ${OUT}/${KIND}.out
exit ${rc}
