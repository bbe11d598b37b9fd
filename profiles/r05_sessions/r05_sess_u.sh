# r05 session u: fp32 k_postpre_lds -- branch vs select check sums at 2 / 3 register sets of
# loads in flight (PGMG_CHK_SEL, PGMG_F32_DEPTH); fp64 branch vs select again
set -u
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 500 python -u scripts/pp_ab.py --dtype f32 --rounds 4 b_d3=$P/libpgmg_f32pk1.so s_d2=$P/libpgmg_s2d2.so b_d2=$P/libpgmg_bd2.so > $O/ab_f32.jsonl 2> $O/ab.err || exit $?
timeout -k 10 400 python -u scripts/pp_ab.py --rounds 4 b=$P/libpgmg_f32pk1.so s=$P/libpgmg_chk2.so > $O/ab_f64.jsonl 2>> $O/ab.err || exit $?
