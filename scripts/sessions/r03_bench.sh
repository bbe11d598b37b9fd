#!/bin/bash
# r03: bench.py as the driver runs it (--warmup 5 --steps 20) and rocprofv3 kernel statistics
# of the headline leg of the same command.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --other-configs off --dropin off --general-rhs off --fast-mode off --pmc off > gpurun_out/prof.log 2>&1 || exit $?
echo done
