set -o pipefail
O=gpurun_out/r02_ppb2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/pp_ab.py --n 16385 --rounds 4 b3072=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so b3584=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PP_BLOCKS=3584 b4096=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PP_BLOCKS=4096 > $O/ab.jsonl 2>&1; rc=$?; cut -c1-100 $O/ab.jsonl; exit $rc
