set -o pipefail
mkdir -p gpurun_out
export PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
run() { # N worlds blocks
  if [ "$3" = d ]; then unset PGMG_PP_BLOCKS; else export PGMG_PP_BLOCKS=$3; fi
  timeout -k 10 200 python scripts/strip_probe.py --n $1 --worlds $2 --steps 10 --warmup 2 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('N=$1 blocks=$3', 'W=%d r=%d' % (d['world'], d['rank']), d['ms_per_cycle'])" || exit 1
}
for rep in 1 2; do
for b in d 6144 9216 12288; do run 32769 1 $b; done
for b in d 1024 1536 2048; do run 32769 8 $b; done
for b in d 768 1024; do run 16385 4 $b; done
done
