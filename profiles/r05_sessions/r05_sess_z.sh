# r05 session z: bench.py's multi-rank paths on the current tree (one-GPU box): the driver's
# launcher shape with SOLO ranks (null transport), and real messages through host memory
set -u
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
PGMG_BENCH_SOLO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/solo2.out 2> $O/solo2.err || exit $?
PGMG_BENCH_TRANSPORT=host timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/host2.out 2> $O/host2.err || exit $?
