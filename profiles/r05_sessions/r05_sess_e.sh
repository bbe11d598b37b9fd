# r05 session e: in-place op tests (both deferral forms), op A/B, fp32 k_postpre variants
set -u
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread > $O/tests_ops.log 2>&1 || exit $?
PGMG_LIB=$L/libpgmg_ab.so PGMG_OPIP_BAR=0 PGMG_OP2IP_BAR=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread -k jacobi > $O/tests_ops_nobar.log 2>&1 || exit $?
PGMG_LIB=$L/libpgmg_ab.so timeout -k 10 300 python -u scripts/op_ip_ab.py --rounds 2 > $O/op_ip_ab.jsonl 2> $O/op_ip_ab.err || exit $?
timeout -k 10 600 python -u scripts/pp_ab.py --dtype f32 --rounds 3 \
  base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_base.so \
  qnone=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_qnone.so \
  qall=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so \
  qd2=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_qd2.so \
  qload=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_qload.so \
  qstore=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_qstore.so \
  qrowonly=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_qrowonly.so > $O/pp_f32.jsonl 2> $O/pp_f32.err || exit $?
