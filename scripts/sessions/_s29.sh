set -o pipefail
O=gpurun_out/r02_small
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/pp_ab.py --n 16385 --rounds 3 d8192=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so p4096=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_FUSED_SMALL_PTS=4096 p2048=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_FUSED_SMALL_PTS=2048 p4096m512=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_FUSED_SMALL_PTS=4096,PGMG_FUSED_SMALL_MIN=512 > $O/ab.jsonl 2>&1; rc=$?; cut -c1-150 $O/ab.jsonl; exit $rc
