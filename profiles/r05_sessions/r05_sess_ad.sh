# r05 session ad: fp32 k_postpre_lds grid (PGMG_PP_BLOCKS) re-checked with the packed stages
set -u
export TMPDIR=/tmp
O=gpurun_out/r05ad; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 500 python -u scripts/pp_ab.py --dtype f32 --rounds 3 b3072=$L b2048=$L:PGMG_PP_BLOCKS=2048 b2560=$L:PGMG_PP_BLOCKS=2560 b4096=$L:PGMG_PP_BLOCKS=4096 b6144=$L:PGMG_PP_BLOCKS=6144 > $O/ab_f32_grid.jsonl 2> $O/ab.err || exit $?
