# r05 session l: the tail's top level per cycle kind -- V at 16385 / 4097 and W at 4097 with the
# tail from 65 (default) and from 33
set -u
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
L=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so
timeout -k 10 600 python -u scripts/pp_ab.py --n 4097 --steps 40 --rounds 3 t65=$L t33=$L:AB_TAIL_N=33 > $O/v4097.jsonl 2> $O/v4097.err || exit $?
timeout -k 10 600 python -u scripts/pp_ab.py --n 16385 --steps 20 --rounds 3 t65=$L t33=$L:AB_TAIL_N=33 > $O/v16385.jsonl 2> $O/v16385.err || exit $?
timeout -k 10 600 python -u scripts/pp_ab.py --n 4097 --kind W --steps 4 --rounds 2 t65=$L t33=$L:AB_TAIL_N=33 > $O/w4097.jsonl 2> $O/w4097.err || exit $?
