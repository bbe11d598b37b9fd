#!/bin/bash
# A/B of library builds on F-cycles at 16385: bash scripts/ab_libF.sh lib1.so lib2.so ...
set -u
for rep in 1 2 3; do
  for L in "$@"; do
    PGMG_LIB=$PWD/$L timeout -k 10 200 python bench.py --cycle F --steps 10 --warmup 2 --cpu-baseline off | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); print('$L', d['value'])" || exit 1
  done
done
