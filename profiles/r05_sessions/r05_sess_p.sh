# r05 session p: the finest pass's check residuals' cost (measurement build with the checks'
# residuals replaced by the iterate: phi unchanged at 16385, the level-0 checks never fire)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
P=parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 600 python -u scripts/pp_ab.py --rounds 4 base=$P/libpgmg_ab.so cheap=$P/libpgmg_cheapchk.so fast=$P/libpgmg_ab.so:AB_FLAGS=4096 > $O/pp.jsonl 2> $O/pp.err || exit $?
