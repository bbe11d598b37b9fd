set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 900 python scripts/pp_ab.py --rounds 2 p0=$L p1=$L:PGMG_PITCH_PAD16=1 p4=$L:PGMG_PITCH_PAD16=4 p32=$L:PGMG_PITCH_PAD16=32 p247=$L:PGMG_PITCH_PAD16=247 \
  b0=$L:PGMG_PP_BLOCKS=512 b1=$L:PGMG_PP_BLOCKS=512,PGMG_PITCH_PAD16=1 b4=$L:PGMG_PP_BLOCKS=512,PGMG_PITCH_PAD16=4 b32=$L:PGMG_PP_BLOCKS=512,PGMG_PITCH_PAD16=32 b247=$L:PGMG_PP_BLOCKS=512,PGMG_PITCH_PAD16=247 > gpurun_out/ab10.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab10.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:6s} r{d['round']} pp {d['pp']:.4f} pre {d['pre']:.4f} post {d['post']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
