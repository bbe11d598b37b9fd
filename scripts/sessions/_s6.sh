set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 900 python scripts/pp_ab.py --rounds 3 new=$L/libpgmg.so ab0=$L/libpgmg_ab.so \
  r14=$L/libpgmg_ab.so:PGMG_REV=16384 r13=$L/libpgmg_ab.so:PGMG_REV=$(( (1<<13) | (1<<29) )) \
  ralt=$L/libpgmg_ab.so:PGMG_REV=713042560 > gpurun_out/ab6.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab6.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:10s} r{d['round']} pp {d['pp']:.4f} pre {d['pre']:.4f} post {d['post']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
