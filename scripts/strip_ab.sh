#!/bin/bash
# Interleaved A/B of launch-geometry knobs (measurement build) on one SOLO rank of W = 8 at
# N = 16385: scripts/strip_ab.sh "name:VAR=v;VAR2=w" ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
for round in 1 2; do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    ( IFS=';'; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      PGMG_LIB=$LIB timeout -k 10 200 python3 scripts/strip_probe.py --worlds 8 --steps 40 2>/dev/null | sed "s/^/{\"variant\": \"$name\", \"round\": $round, \"r\": /; s/\$/}/" ) || exit $?
  done
done
