# r05 session w: k_post's check sums as selects (PGMG_CHK_SEL_LV=3, fp64) -- V at 16385 / 4097,
# F at 16385, interleaved
set -u
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 300 python -u scripts/pp_ab.py --rounds 3 lv0=$P/libpgmg_lv0.so lv3=$P/libpgmg_lv3.so > $O/ab_v16385.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python -u scripts/pp_ab.py --kind F --rounds 3 lv0=$P/libpgmg_lv0.so lv3=$P/libpgmg_lv3.so > $O/ab_f16385.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 300 python -u scripts/pp_ab.py --n 4097 --steps 40 --rounds 3 lv0=$P/libpgmg_lv0.so lv3=$P/libpgmg_lv3.so > $O/ab_v4097.jsonl 2>> $O/ab.err || exit $?
