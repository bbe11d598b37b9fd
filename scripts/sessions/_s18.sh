set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fcycle.py tests/test_gpu_spec.py tests/test_gpu_strips.py tests/test_gpu_fp32.py tests/test_gpu_wtail.py tests/test_gpu_strips_fcycle.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t18.log 2>&1; rc=$?; tail -3 gpurun_out/t18.log; [ $rc -eq 0 ] || exit $rc
PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so timeout -k 10 200 python scripts/tail_prof.py 4097 > gpurun_out/tail_prof5.jsonl 2>&1 || exit 1; grep -v amdgpu gpurun_out/tail_prof5.jsonl | head -2
for L in libpgmg_base.so libpgmg.so libpgmg_base.so libpgmg.so; do PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/$L timeout -k 10 200 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off --general-rhs off --pmc off > gpurun_out/bw.log 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/bw.log').read().strip().splitlines()[-1]); print('$L', d['value'], d['ms_per_step'])"; done
