#!/bin/bash
# r06 GPU session: the carry's tests first (verbose), smoke(), the whole GPU suite, then the
# driver-shaped bench line.  bash scripts/r06_session.sh OUT [STEPS...]
# STEPS (default: carry smoke tests bench): any of carry smoke tests bench solo2 solo8 host2 carry_ab stagger levels
# Each GPU step runs under its own time limit; a time limit (124/137), an abort (134) or a
# fault (139) ends the session.
set -u
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r06}
shift || true
STEPS=${*:-carry smoke tests bench}
mkdir -p ${OUT}
step() {   # step NAME LIMIT CMD... (stdout -> OUT/NAME.out, stderr -> OUT/NAME.err)
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] ${name}" >&2
  timeout -k 10 ${lim} "$@" > ${OUT}/${name}.out 2> ${OUT}/${name}.err
  local rc=$?
  echo "[$(date +%T)] ${name} rc=${rc}" >&2
  tail -2 ${OUT}/${name}.out >&2
  case ${rc} in
    124|134|137|139) echo "stopping after ${name} (rc ${rc})" >&2; exit ${rc} ;;
  esac
  return 0
}
for s in ${STEPS}; do
  case ${s} in
    carry) step carry 600 python -u -m pytest tests/test_gpu_carry.py -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py --gpus 1 --warmup 5 --steps 20 --save-profiles ${OUT}/prof ;;
    bench_F) step bench_F 300 python bench.py --cycle F --warmup 2 --steps 20 --cpu-baseline off --pmc off --trace off ;;
    bench_W) step bench_W 300 python bench.py --cycle W --n 4097 --warmup 2 --steps 10 --cpu-baseline off --pmc off --trace off ;;
    bench_f32) step bench_f32 400 python bench.py --dtype f32 --warmup 5 --steps 20 --cpu-baseline off --save-profiles ${OUT}/prof_f32 ;;
    solo2) step solo2 300 env PGMG_BENCH_SOLO=1 python bench.py --gpus 2 --warmup 2 --steps 10 --reps 2 ;;
    solo8) step solo8 400 env PGMG_BENCH_SOLO=1 python bench.py --gpus 8 --warmup 2 --steps 10 --reps 2 ;;
    host2) step host2 400 env PGMG_BENCH_TRANSPORT=host python bench.py --gpus 2 --warmup 2 --steps 5 --reps 2 ;;
    stagger) step stagger 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python scripts/stagger_probe.py --staggers ${STAGGERS:-0,4096,65536,1048576} ;;
    variants) step variants 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python scripts/stagger_probe.py --reps 5 --variants "${VARIANTS}" ;;
    ctrace) step ctrace 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/ctrace -o run -- python3 scripts/carry_trace.py && step ctrace_an 60 python3 scripts/carry_trace.py --analyse ${OUT}/ctrace ;;
    order) step order1 300 python3 scripts/order_probe.py --order ncnc && step order2 300 python3 scripts/order_probe.py --order cncn && step order3 300 python3 scripts/order_probe.py --order ncnc --dummy-gib 24 ;;
    order2) step warm 300 python3 scripts/order_probe.py --order n --reps 30 && step keep 300 python3 scripts/order_probe.py --order nnn --keep ;;
    contig) step contig1 300 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so PGMG_CONTIG=1 python3 scripts/order_probe.py --order ncnc && step contig2 300 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so PGMG_CONTIG=1 python3 scripts/order_probe.py --order nnn --keep && step contig0 300 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/order_probe.py --order ncnc ;;
    shuffle) for mb in ${SHUFFLE_MB:-2 64}; do step shuffle${mb} 300 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so PGMG_SHUFFLE_MB=${mb} python3 scripts/order_probe.py --order ncnc; done ;;
    shuffle_rep) for i in 1 2 3; do step shuffle_rep${i} 300 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so PGMG_SHUFFLE_MB=${SHUFFLE_MB:-2} python3 scripts/order_probe.py --order ncnc; done ;;
    strace) step strace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d ${OUT}/strace -o run -- python3 scripts/single_call_trace.py && step strace_an 60 python3 scripts/single_call_trace.py --analyse ${OUT}/strace ;;
    carry_ab) step carry_ab 400 python scripts/carry_ab.py --rounds 3 ;;
    spin_ab) step spin_ab 400 python scripts/carry_ab.py --rounds 3 --variants carry,no_spin ;;
    band) step band 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/band_probe.py --values ${BANDS:-0,1024,1536,2048} --rounds 2 ;;
    ppblocks) step ppblocks 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/band_probe.py --knob PGMG_PP_BLOCKS --values ${PPB:-0,1536,2048,2560,3584,4096} --rounds 2 ;;
    ppxcd) step ppxcd 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/band_probe.py --knob PGMG_PP_XCD --values 0,1,0,1 --rounds 2 ;;
    fusedxcd) step fusedxcd 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/band_probe.py --knob PGMG_FUSED_XCD --values 0,1,0,1 --rounds 2 ;;
    fxcd) step fxcd 600 env PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_probe.so python3 scripts/band_probe.py --cycle F --knob PGMG_F_XCD --values 0,off,0,off --rounds 2 ;;
    wtrace) step wtrace 300 rocprofv3 --kernel-trace --output-format csv -d ${OUT}/wtrace -o run -- python3 scripts/w_trace.py && step wtrace_an 60 python3 scripts/w_trace.py --analyse ${OUT}/wtrace ;;
    levels) step levels 300 python scripts/level_pmc.py run --n 16385 --out ${OUT}/levels ;;
    *) echo "unknown step ${s}" >&2 ;;
  esac
done
