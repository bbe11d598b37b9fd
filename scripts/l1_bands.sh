#!/bin/bash
# Level-1 band height A/B: per-kernel rocprofv3 kernel traces of a 10-cycle
# V call at N = 16385 with the big levels' workgroup target PGMG_FUSED_BLOCKS (measurement build
# libpgmg_ab.so) at 3072 (default: 25 coarse rows = 50 fine rows per level-1 band, 8 halo rows
# in k_pre), 2048, 1536 and 1024 (taller bands: 64 / 86 / 128 fine rows), then an interleaved
# V-cycles/s A/B of the same variants.   bash scripts/l1_bands.sh OUT
set -u
export TMPDIR=/tmp
OUT=${1:-gpurun_out/l1_bands}
mkdir -p ${OUT}
export PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
for b in 3072 2048 1536 1024; do
  PGMG_FUSED_BLOCKS=${b} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/tl_${b} -o run -- python3 scripts/cycle_timeline.py --child --n 16385 --cycles 10 > ${OUT}/tl_${b}.log 2>&1 || exit $?
  python3 scripts/cycle_timeline.py --parse ${OUT}/tl_${b} --cycles 10 > ${OUT}/tl_${b}.json || exit $?
  rm -rf ${OUT}/tl_${b}
done
timeout -k 10 600 python3 scripts/ab_env.py --rounds 3 --grids V16385,V4097 \
  "b3072:" "b2048:PGMG_FUSED_BLOCKS=2048" "b1536:PGMG_FUSED_BLOCKS=1536" "b1024:PGMG_FUSED_BLOCKS=1024" \
  > ${OUT}/ab.jsonl 2> ${OUT}/ab.err || exit $?
cat ${OUT}/ab.jsonl
