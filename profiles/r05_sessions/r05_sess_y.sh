# r05 session y: which bulk-level visits of the FMG start + W-cycle at 32769 fire (W plan trace
# of the measurement build), and the same for W calls at 4097
set -u
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
export PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so
PGMG_SPEC_TRACE=1 timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import torch, _pkgload
pg = _pkgload.load()
with pg.Solver(32769) as s:
    s.set_problem(); s.fcycle(1); s.sync(); print('F done', s.stats(), file=sys.stderr, flush=True)
    s.wcycle(1); s.sync(); print('W done', s.stats(), s.dist_info(), s.solution_hash(0), file=sys.stderr, flush=True)
" > $O/g32769.out 2> $O/g32769.err || exit $?
