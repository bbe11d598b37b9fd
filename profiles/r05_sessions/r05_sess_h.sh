# r05 session h: in-place op tests, op A/B (in place vs ping-pong), kernel trace of the op calls
set -u
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread > $O/tests_ops.log 2>&1 || exit $?
PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so timeout -k 10 300 python -u scripts/op_ip_ab.py --quick --rounds 3 > $O/op_ip_ab.jsonl 2> $O/op_ip_ab.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/opprof -o run -- python3 scripts/op_ip_ab.py --quick --rounds 1 > $O/opprof.log 2>&1 || exit $?
