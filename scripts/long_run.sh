#!/bin/bash
# V-cycles/s over long runs (levels above the tail reach eps and decide in-stream; their
# fix-ups fire) for env-knob variants:  bash scripts/long_run.sh N STEPS "VAR=v" ...
set -u
N=$1; STEPS=$2; shift 2
for cfg in "$@"; do
  (export $cfg; timeout -k 10 200 python bench.py --n $N --steps $STEPS --warmup 5 --cpu-baseline off --timing graph) | python -c "import sys,json; d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); print('$cfg', 'N=$N steps=$STEPS', d['value'])" || exit 1
done
