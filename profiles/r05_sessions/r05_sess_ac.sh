# r05 session ac: bench.py --gpus 8 through the host-staged transport (8 rank processes on the one
# GPU, real messages through host memory): the N = 8 launch path and both grids' parity
set -u
export TMPDIR=/tmp
O=gpurun_out/r05ac; mkdir -p $O
PGMG_BENCH_TRANSPORT=host timeout -k 10 800 python bench.py --gpus 8 --steps 3 --warmup 1 > $O/host8.out 2> $O/host8.err || exit $?
