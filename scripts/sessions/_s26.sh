set -o pipefail
O=gpurun_out/r02_tres
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wtail.py tests/test_gpu_parity.py tests/test_gpu_fcycle.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/pp_ab.py --kind W --n 4097 --steps 5 --rounds 3 base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_tbase.so new=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_tnew.so > $O/ab_w.jsonl 2>&1; rc=$?; cut -c1-200 $O/ab_w.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/pp_ab.py --kind V --n 16385 --rounds 2 base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_tbase.so new=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_tnew.so > $O/ab_v.jsonl 2>&1; rc=$?; cut -c1-200 $O/ab_v.jsonl; exit $rc
