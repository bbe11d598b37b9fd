#!/bin/bash
# r03 session: per-level rocprofv3 table of a V-cycle at 16385 on the final tree
set -u
export TMPDIR=/tmp
O=gpurun_out/r03_levels
mkdir -p $O
timeout -k 10 700 python scripts/level_pmc.py run --out $O/levels > $O/levels.jsonl 2>&1; rc=$?; cut -c1-400 $O/levels.jsonl; exit $rc
