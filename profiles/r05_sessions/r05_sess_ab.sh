# r05 session ab: k_postpre_lds without the per-step scheduling fence (PGMG_NO_STEP_SCHED), fp64
# and fp32, interleaved
set -u
export TMPDIR=/tmp
O=gpurun_out/r05ab; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 300 python -u scripts/pp_ab.py --rounds 4 base=$P/libpgmg_base.so nss=$P/libpgmg_nss.so > $O/ab_f64.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python -u scripts/pp_ab.py --dtype f32 --rounds 3 base=$P/libpgmg_base.so nss=$P/libpgmg_nss.so > $O/ab_f32.jsonl 2>> $O/ab.err || exit $?
