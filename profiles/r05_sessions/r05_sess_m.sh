# r05 session m: fp32 k_postpre_lds grid and prefetch depth (4 waves per SIMD: 1024 resident)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
L=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
D2=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_f32d2.so
timeout -k 10 900 python -u scripts/pp_ab.py --dtype f32 --rounds 3 \
  b3072=$L b2048=$L:PGMG_PP_BLOCKS=2048 b4096=$L:PGMG_PP_BLOCKS=4096 b6144=$L:PGMG_PP_BLOCKS=6144 \
  b1024=$L:PGMG_PP_BLOCKS=1024 d2=$D2 d2b4096=$D2:PGMG_PP_BLOCKS=4096 > $O/f32grid.jsonl 2> $O/f32grid.err || exit $?
