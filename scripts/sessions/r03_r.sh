#!/bin/bash
# r03 session: bench.py's F-cycle (N = 16385) and W-cycle (N = 4097) lines on the final tree
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --cycle F --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/bench_F.log 2>&1 || { tail -5 gpurun_out/bench_F.log; exit 1; }
grep '^{' gpurun_out/bench_F.log | cut -c1-300
timeout -k 10 600 python bench.py --cycle W --N 4097 --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/bench_W.log 2>&1 || { tail -5 gpurun_out/bench_W.log; exit 1; }
grep '^{' gpurun_out/bench_W.log | cut -c1-300
