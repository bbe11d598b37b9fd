#!/bin/bash
# Per-level kernel durations of one rank's strip work (PGMG_FLAG_SOLO) for env-knob variants.
#   bash scripts/strip_level_sweep.sh WORLD "VAR=v" "VAR=v2 VAR2=w" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
W=$1; shift
i=0
for cfg in "$@"; do
  d=gpurun_out/sls_$i
  rm -rf $d
  echo "=== $i W=$W $cfg"
  (export $cfg; timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 scripts/strip_probe.py --worlds $W --steps 10 > $d.log 2>&1) || { echo "FAILED $cfg"; exit 1; }
  grep '^{' $d.log
  python3 scripts/level_summary.py $d "$cfg"
  i=$((i+1))
done
