#!/bin/bash
# A/B of library builds: bash scripts/ab_lib.sh lib1.so lib2.so ...  (bench V at 16385, interleaved x3)
set -u
for rep in 1 2 3; do
  for L in "$@"; do
    PGMG_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-baseline off | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); print('$L', d['value'], d['roofline']['ms_per_launch'])" || exit 1
  done
done
