set -o pipefail
O=gpurun_out/r02_l1a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1post.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -25 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/pp_ab.py --n 16385 --rounds 3 base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so l1=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so:AB_FLAGS=8192 > $O/ab.jsonl 2>&1; rc=$?; cat $O/ab.jsonl; exit $rc
