#!/bin/bash
# r04 coarse-end measurements (GPU box): per-kernel V-cycle timelines at N = 16385 and 4097 with
# the small levels as 2D LDS tiles (default) and as row-marching passes (PGMG_FLAG_NO_CTILE =
# 65536), and the strips' per-rank compute (SOLO ranks: W = 1, 2, 4, 8; the timeline of rank 4 of
# W = 8).  Each step under its own time limit; the first failure ends the session.
set -u
export TMPDIR=/tmp
OUT=${1:-gpurun_out/coarse}
mkdir -p ${OUT}
for n in 16385 4097; do
  for fl in 0 65536; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/tl_${n}_${fl} -o run -- python3 scripts/cycle_timeline.py --child --n ${n} --cycles 10 --flags ${fl} > ${OUT}/tl_${n}_${fl}.log 2>&1 || exit $?
    python3 scripts/cycle_timeline.py --parse ${OUT}/tl_${n}_${fl} --cycles 10 > ${OUT}/tl_${n}_${fl}.json || exit $?
    rm -rf ${OUT}/tl_${n}_${fl}
  done
done
timeout -k 10 300 python3 scripts/strip_probe.py --n 16385 > ${OUT}/strip_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/st8 -o run -- python3 scripts/cycle_timeline.py --child --n 16385 --world 8 --rank 4 > ${OUT}/st8.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse ${OUT}/st8 > ${OUT}/timeline_W8_rank4.json || exit $?
rm -rf ${OUT}/st8
cat ${OUT}/strip_probe.jsonl
