#!/bin/bash
# r03 session: the multi-process bench harness on the one-GPU box (ranks share device 0):
# null transport (timing harness) at 2 and 4 ranks, host-staged transport at 2 (parity)
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for n in 2 4; do
  PGMG_BENCH_SOLO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/solo_$n.log 2>&1 || { tail -20 gpurun_out/solo_$n.log; exit 1; }
  grep '^{' gpurun_out/solo_$n.log | cut -c1-300
done
PGMG_BENCH_TRANSPORT=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --N 4097 --steps 10 --warmup 3 > gpurun_out/hostmp_2.log 2>&1 || { tail -20 gpurun_out/hostmp_2.log; exit 1; }
grep '^{' gpurun_out/hostmp_2.log | cut -c1-400
