set -o pipefail
O=gpurun_out/r02_xcd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/pp_ab.py --n 16385 --rounds 4 ab=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so xcd=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_xcd.so > $O/ab.jsonl 2>&1; rc=$?; cut -c1-140 $O/ab.jsonl; exit $rc
