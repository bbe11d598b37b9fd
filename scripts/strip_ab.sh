#!/bin/bash
# Strip geometry A/B (r04): one SOLO rank of a W = 8 strip job at N = 16385 (scripts/strip_probe.py,
# rank 0 and a middle rank), the measurement build's band knobs varied for the thin distributed
# levels (PGMG_FUSED_SMALL_PTS: fine points per workgroup below 2^23 points, default 8192;
# PGMG_FUSED_SMALL_MIN: at least this many workgroups, default 256), two interleaved rounds.
#   bash scripts/strip_ab.sh OUT
set -u
OUT=${1:-gpurun_out/strip_ab}
mkdir -p ${OUT}
export PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
for round in 0 1; do
  for v in "base:" "pts4096:PGMG_FUSED_SMALL_PTS=4096" "pts2048:PGMG_FUSED_SMALL_PTS=2048" \
           "min512:PGMG_FUSED_SMALL_MIN=512" "min1024:PGMG_FUSED_SMALL_MIN=1024"; do
    name=${v%%:*}
    envs=${v#*:}
    env ${envs} timeout -k 10 200 python3 scripts/strip_probe.py --worlds 8 --steps 30 \
      > ${OUT}/${name}_r${round}.jsonl 2> ${OUT}/${name}_r${round}.err || exit $?
    echo "${name} r${round}: $(tr '\n' ' ' < ${OUT}/${name}_r${round}.jsonl)"
  done
done
