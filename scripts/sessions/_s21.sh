set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 600 python scripts/pp_ab.py --rounds 3 d=$L f1536=$L:PGMG_FUSED_BLOCKS=1536 f2048=$L:PGMG_FUSED_BLOCKS=2048 f4096=$L:PGMG_FUSED_BLOCKS=4096 f6144=$L:PGMG_FUSED_BLOCKS=6144 > gpurun_out/ab21.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab21.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:6s} r{d['round']} pp {d['pp']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
