#!/bin/bash
# Per-level kernel durations (rocprofv3 kernel trace) of the V-cycle for env-knob variants.
#   bash scripts/level_sweep.sh "PGMG_FUSED_BLOCKS=1536" "PGMG_FUSED_BLOCKS=2304" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  d=gpurun_out/ls_$i
  rm -rf $d
  echo "=== $i $cfg"
  env $cfg > /dev/null   # validate
  (export $cfg; timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > $d.log 2>&1) || { echo "FAILED $cfg"; exit 1; }
  python3 scripts/level_summary.py $d "$cfg"
  i=$((i+1))
done
