#!/bin/bash
# SQ issue/wait counters of the V-cycle kernels (one rocprofv3 --pmc pass, kernel trace only)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/pmc_sq.log 2>&1
