set -o pipefail
mkdir -p gpurun_out
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 600 python scripts/pp_ab.py --rounds 3 new=$L/libpgmg.so occ3=$L/libpgmg_occ3.so > gpurun_out/ab17.log 2>&1; rc=$?
python - <<'P'
import json
for l in open('gpurun_out/ab17.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f"{d['variant']:6s} r{d['round']} pp {d['pp']:.4f} cyc {d['ms_cycle']:.4f} parity {d['parity']}")
    else: print(l.rstrip()[:200])
P
exit $rc
