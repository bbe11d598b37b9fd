set -o pipefail
O=gpurun_out/r02_robust
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust_rhs.py tests/test_oracle_mt_rhs.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 14 $O/tests.log; exit $rc
