set -o pipefail
O=gpurun_out/r02_nos
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python scripts/pp_ab.py --n 16385 --rounds 4 ab=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so nosched=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_nos.so > $O/ab.jsonl 2>&1; rc=$?; cut -c1-120 $O/ab.jsonl; exit $rc
