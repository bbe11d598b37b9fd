# r05 session r: out-of-place op kernels' launch forms (residual in 512-thread workgroups,
# restriction / prolongation grids)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$L PGMG_OPR_NTH=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k residual --timeout 120 --timeout-method thread > $O/tests_r512.log 2>&1 || exit $?
PGMG_LIB=$L timeout -k 10 400 python -u scripts/op_misc_ab.py --rounds 3 base r512:PGMG_OPR_NTH=512 r512b1024:PGMG_OPR_NTH=512,PGMG_OPR_BLOCKS=1024 \
  rs1024:PGMG_OPRS_BLOCKS=1024 rs2048:PGMG_OPRS_BLOCKS=2048 p1024:PGMG_OPP_BLOCKS=1024 p2048:PGMG_OPP_BLOCKS=2048 p8192:PGMG_OPP_BLOCKS=8192 > $O/ab.jsonl 2> $O/ab.err || exit $?
