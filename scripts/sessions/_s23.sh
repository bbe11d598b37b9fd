set -o pipefail
O=gpurun_out/r02_l1b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python scripts/pp_ab.py --n 16385 --rounds 2 base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so l1=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so:AB_FLAGS=8192 l1_nomask=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_l1m.so:AB_FLAGS=8192 l1_nostage=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_l1s.so:AB_FLAGS=8192 l1_d3=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_l1d3.so:AB_FLAGS=8192 > $O/ab.jsonl 2>&1; rc=$?; cat $O/ab.jsonl; exit $rc
