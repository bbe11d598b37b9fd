#!/bin/bash
# r03 session: the host-code sanitizer runs (tests/test_gpu_sanitize.py)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sanitize.py -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/san_tests.log 2>&1
rc=$?; tail -25 gpurun_out/san_tests.log; exit $rc
