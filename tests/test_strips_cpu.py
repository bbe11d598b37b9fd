"""CPU: the row-strip decomposition plan and the multi-rank bootstrap (gloo, world 2).

The plan is the host arithmetic every rank runs in pgmg_create (pgmg_plan_strips):
strips must tile the grid, split points must be multiples of 2^Ld so every
distributed level halves evenly (coarse row jc on the rank owning fine row 2jc).
"""
import os
import socket

import pytest


def _plans(pg, N, world, tail_n=65, gather_n=1025):
    return [pg.plan_strips(N, world, r, tail_n, gather_n) for r in range(world)]


@pytest.mark.parametrize("N", [513, 1025, 4097, 16385, 32769])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("gather_n", [65, 257, 1025])
def test_strips_tile_the_grid(pgmg, N, world, gather_n):
    plans = _plans(pgmg, N, world, gather_n=gather_n)
    nd = {p[2] for p in plans}
    assert len(nd) == 1
    Ld = nd.pop()
    if Ld == 0:  # replicas: every rank holds the whole grid
        assert all(p[:2] == (0, N) for p in plans)
        return
    assert plans[0][0] == 0 and plans[-1][1] == N
    for a, b in zip(plans, plans[1:]):
        assert a[1] == b[0]
    for lo, hi, _ in plans:
        assert lo % (1 << Ld) == 0
        assert hi - lo >= 16 << (Ld - 1)
    # every distributed level has N_l > gather_n
    assert (N - 1) // (1 << (Ld - 1)) + 1 > gather_n


def test_default_plan_16385_8_ranks(pgmg):
    plans = _plans(pgmg, 16385, 8)
    assert [p[:2] for p in plans][:2] == [(0, 2048), (2048, 4096)]
    assert plans[0][2] == 4   # 16385, 8193, 4097, 2049 split; 1025 and below on rank 0


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import _pkgload
    pg = _pkgload.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # the bench.py bootstrap: rank 0 makes the RCCL unique id, gloo broadcasts it
    t = torch.tensor(list(pg.unique_id()) if rank == 0 else [0] * 128, dtype=torch.uint8)
    dist.broadcast(t, 0)
    ids = [torch.zeros(128, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(ids, t)
    lo, hi, nd = pg.plan_strips(16385, world, rank)
    plans = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(plans, torch.tensor([lo, hi, nd]))
    # the max-over-ranks timing reduction bench.py performs
    tt = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((all(bool((i == ids[0]).all()) for i in ids), [p.tolist() for p in plans],
               float(tt.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_bootstrap_and_plan():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    same_id, plans, tmax = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same_id
    assert plans == [[0, 8192, 4], [8192, 16385, 4]]
    assert tmax == 2.0
