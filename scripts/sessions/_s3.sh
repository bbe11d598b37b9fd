set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python scripts/pp_ab.py --rounds 2 base=$L/libpgmg_base.so new=$L/libpgmg.so \
  ab512=$L/libpgmg_ab.so:PGMG_PP_BLOCKS=512 ab1024=$L/libpgmg_ab.so:PGMG_PP_BLOCKS=1024 ab1536=$L/libpgmg_ab.so:PGMG_PP_BLOCKS=1536 \
  d6_512=$L/libpgmg_dma6.so:PGMG_PP_BLOCKS=512 d6_1024=$L/libpgmg_dma6.so:PGMG_PP_BLOCKS=1024 d6_1536=$L/libpgmg_dma6.so:PGMG_PP_BLOCKS=1536 d6_3072=$L/libpgmg_dma6.so \
  d4_512=$L/libpgmg_dma4.so:PGMG_PP_BLOCKS=512 d4_1536=$L/libpgmg_dma4.so:PGMG_PP_BLOCKS=1536 d4_3072=$L/libpgmg_dma4.so > gpurun_out/ab3.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab3.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:10s} r{d['round']} pp {d['pp']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
