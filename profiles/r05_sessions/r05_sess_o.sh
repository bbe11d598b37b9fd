# r05 session o: the deferred scatter's forms (partial writes / whole 64-byte segments) and grid,
# kernel-traced; the op tests with the whole-segment form
set -u
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_LIB=$L PGMG_SCAT_FULL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k jacobi --timeout 120 --timeout-method thread > $O/tests_full.log 2>&1 || exit $?
for v in "all:" "full:PGMG_SCAT_FULL=1" "per16:PGMG_SCAT_PER=16" "full16:PGMG_SCAT_FULL=1,PGMG_SCAT_PER=16" "per64:PGMG_SCAT_PER=64" "full64:PGMG_SCAT_FULL=1,PGMG_SCAT_PER=64"; do
  n=${v%%:*}; e=$(echo ${v#*:} | tr ',' ' ')
  env PGMG_LIB=$L $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 scripts/op_ip_ab.py --only-inplace --rounds 1 > $O/$n.log 2>&1 || exit $?
done
