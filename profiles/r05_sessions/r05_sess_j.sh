# r05 session j: the tail's W visits merged into one launch -- W / F / spec GPU tests, then
# BASELINE configs[4]'s W call with and without the merge
set -u
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "wcycle or wtail or W or fmg or config4 or spec" -x -q --timeout 300 --timeout-method thread > $O/tests_w.log 2>&1; rc=$?
echo "rc=$rc" >> $O/tests_w.log
case $rc in 0|1) ;; *) exit $rc;; esac
PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so timeout -k 10 600 python -u scripts/fmgw_time.py --rounds 2 merged:PGMG_TAIL_VISITS=1 split:PGMG_TAIL_VISITS=0 > $O/fmgw.jsonl 2> $O/fmgw.err || exit $?
bash scripts/r05_sess_i.sh || exit $?
