# r05 session t: k_postpre_lds check sums as selects instead of a branch (PGMG_CHK_SEL):
# fp32 (packed stages) and fp64 interleaved A/Bs, fp32 tests on the select build
set -u
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
PGMG_LIB=$P/libpgmg_chk1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32.py -q -x --timeout 120 --timeout-method thread > $O/tests_f32_chk1.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/pp_ab.py --dtype f32 --rounds 3 chk0=$P/libpgmg_f32pk1.so chk1=$P/libpgmg_chk1.so > $O/ab_f32.jsonl 2> $O/ab.err || exit $?
timeout -k 10 400 python -u scripts/pp_ab.py --rounds 3 chk1=$P/libpgmg_chk1.so chk2=$P/libpgmg_chk2.so > $O/ab_f64.jsonl 2>> $O/ab.err || exit $?
