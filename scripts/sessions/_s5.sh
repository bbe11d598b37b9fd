set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python scripts/pp_ab.py --rounds 2 new=$L/libpgmg.so \
  ab504=$L/libpgmg_ab.so:PGMG_PP_BLOCKS=512 ab1008=$L/libpgmg_ab.so:PGMG_PP_BLOCKS=1024 \
  d6_504=$L/libpgmg_dma6.so:PGMG_PP_BLOCKS=512 d6_1008=$L/libpgmg_dma6.so:PGMG_PP_BLOCKS=1024 d6_3072=$L/libpgmg_dma6.so \
  d4_504=$L/libpgmg_dma4.so:PGMG_PP_BLOCKS=512 d4_1008=$L/libpgmg_dma4.so:PGMG_PP_BLOCKS=1024 > gpurun_out/ab5.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab5.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:10s} r{d['round']} pp {d['pp']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
