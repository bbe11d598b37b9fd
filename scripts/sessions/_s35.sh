set -o pipefail
O=gpurun_out/r02_ppb
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/pp_ab.py --n 16385 --rounds 4 b3072=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so b2560=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PP_BLOCKS=2560 b2048=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PP_BLOCKS=2048 b1536=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PP_BLOCKS=1536 > $O/ab.jsonl 2>&1; rc=$?; cut -c1-100 $O/ab.jsonl; exit $rc
