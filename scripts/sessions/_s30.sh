set -o pipefail
O=gpurun_out/r02_robust2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust_rhs.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; grep -E 'PASS|FAIL|rel |passed|failed|Error' $O/tests.log | tail -n 20; exit $rc
