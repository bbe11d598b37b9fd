#!/bin/bash
# Round-end validation session (GPU box): the GPU suite, smoke(), the driver-shaped bench line
# with its rocprofv3 summaries, F- and W-cycle lines and the coarse-end timelines.
#   bash scripts/final_session.sh OUT
# Each GPU step runs under its own time limit.  An ordinary test failure (pytest exit 1) is
# recorded and the session goes on; a time limit (124/137), an abort (134) or a fault (139) ends it.
set -u
export TMPDIR=/tmp
OUT=${1:-gpurun_out/final}
mkdir -p ${OUT}
step() {   # step NAME LIMIT CMD... (stdout -> OUT/NAME.out, stderr -> OUT/NAME.err)
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] ${name}" >&2
  timeout -k 10 ${lim} "$@" > ${OUT}/${name}.out 2> ${OUT}/${name}.err
  local rc=$?
  echo "[$(date +%T)] ${name} rc=${rc}" >&2
  case ${rc} in
    124|134|137|139) echo "stopping after ${name} (rc ${rc})" >&2; exit ${rc} ;;
  esac
  return 0
}
step tests 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --warmup 5 --steps 20 --save-profiles ${OUT}/prof
step bench_F 300 python bench.py --cycle F --warmup 2 --steps 20 --cpu-baseline off --pmc off --trace off
step bench_W 300 python bench.py --cycle W --n 4097 --warmup 2 --steps 10 --cpu-baseline off --pmc off --trace off
step bench_f32 400 python bench.py --dtype f32 --warmup 5 --steps 20 --cpu-baseline off --save-profiles ${OUT}/prof_f32
[ "${SKIP_COARSE:-0}" = 1 ] || step coarse 900 bash scripts/coarse_session.sh ${OUT}/coarse
tail -3 ${OUT}/tests.out >&2
cat ${OUT}/bench.out
