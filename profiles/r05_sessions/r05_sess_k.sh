# r05 session k: configs[1] (3 + 40 V-cycles at 4097) against the latency-bound levels' grids
set -u
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
L=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 900 python -u scripts/pp_ab.py --n 4097 --steps 40 --rounds 3 \
  base=$L fb1024=$L:PGMG_FUSED_BLOCKS=1024 fb2048=$L:PGMG_FUSED_BLOCKS=2048 \
  sp4k=$L:PGMG_FUSED_SMALL_PTS=4096 smin512=$L:PGMG_FUSED_SMALL_MIN=512 \
  pp1024=$L:PGMG_PP_BLOCKS=1024 pp2048=$L:PGMG_PP_BLOCKS=2048 > $O/cfg1.jsonl 2> $O/cfg1.err || exit $?
