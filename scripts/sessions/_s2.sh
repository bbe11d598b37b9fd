set -o pipefail
mkdir -p gpurun_out
P=parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_cross.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_spec.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/pp_ab.py --rounds 3 base=$PWD/$P/libpgmg_base.so new=$PWD/$P/libpgmg.so > gpurun_out/ab2.log 2>&1; rc=$?; cat gpurun_out/ab2.log; exit $rc
