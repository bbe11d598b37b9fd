# r05 session q: the single in-place sweep with 512-thread workgroups (half the column-block
# boundaries): ops tests with it, then the op A/B
set -u
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$L PGMG_OP2IP_NTH=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k jacobi --timeout 120 --timeout-method thread > $O/tests_512.log 2>&1 || exit $?
PGMG_LIB=$L timeout -k 10 300 python -u scripts/op_ip_ab.py --nth --rounds 3 > $O/ab.jsonl 2> $O/ab.err || exit $?
