# r05 session aa: k_post_r2's select-form checks alone (the product default) against none
set -u
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 300 python -u scripts/pp_ab.py --kind F --rounds 3 lv0=$P/libpgmg_lv0.so r2=$P/libpgmg_lvr2.so > $O/ab_f16385.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python -u scripts/pp_ab.py --rounds 3 lv0=$P/libpgmg_lv0.so r2=$P/libpgmg_lvr2.so > $O/ab_v16385.jsonl 2>> $O/ab.err || exit $?
