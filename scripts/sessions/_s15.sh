set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
timeout -k 10 600 python scripts/pp_ab.py --n 4097 --rounds 2 --steps 40 d=$L b1024=$L:PGMG_PP_BLOCKS=1024 b1536=$L:PGMG_PP_BLOCKS=1536 b2048=$L:PGMG_PP_BLOCKS=2048 b3072=$L:PGMG_PP_BLOCKS=3072 b256=$L:PGMG_PP_BLOCKS=256 > gpurun_out/ab15.log 2>&1; rc=$?
timeout -k 10 600 python scripts/pp_ab.py --n 32769 --rounds 1 --steps 5 d=$L b1536=$L:PGMG_PP_BLOCKS=1536 b4608=$L:PGMG_PP_BLOCKS=4608 b6144=$L:PGMG_PP_BLOCKS=6144 >> gpurun_out/ab15.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab15.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:6s} r{d['round']} pp {d['pp']:.4f} pre {d['pre']:.4f} post {d['post']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
