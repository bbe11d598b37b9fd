#!/bin/bash
# One guarded GPU session on the MI355X box (run through gpurun from the repo root).
# Every GPU step has its own time limit; the script stops at the first step that
# faults, aborts, segfaults or times out (anything but exit 0 / pytest's 1).
#   scripts/gpu_session.sh [steps...]   steps: smoke tests bench prof pmc fp32 bench32 sweep ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${*:-smoke tests bench}

run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ;;
    strips) run strips 400 python -m pytest tests/test_gpu_strips.py -m gpu -q -rf -x ;;
    fcycle) run fcycle 600 python -m pytest tests/test_gpu_fcycle.py -m gpu -q -rf ;;
    tests-fast) run tests 600 python -u -m pytest tests -m "gpu and not slow" -v -rf --timeout 200 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
    fp32) run fp32 600 python -m pytest tests/test_gpu_fp32.py -m gpu -q -rf ;;
    bench32) run bench32 600 python bench.py --steps 20 --warmup 3 --dtype f32 --cpu-baseline off ;;
    sweep) run sweep 900 python scripts/fp32_sweep.py --out gpurun_out/fp32_sweep.json ;;
    bench-graph) run bench_graph 600 python bench.py --steps 20 --warmup 3 --timing graph --cpu-baseline off ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off ;;
    bench-quick) run bench_quick 500 python bench.py --steps 20 --warmup 3 --other-configs off --fast-mode off --general-rhs off --pmc off --cpu-baseline off ;;
    t=*) f=${s#t=}; run "t_$(echo "$f" | tr ',/.' '___')" 900 python -u -m pytest ${f//,/ } -m gpu -v -rf --timeout 300 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
