"""Worker functions for the multi-process tests (spawned: importable at module level).

Each worker joins a gloo group on 127.0.0.1 and reports through a queue as (rank, result).
"""
import ctypes as C
import os
import pathlib
import socket
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(target, world, *args, timeout=300):
    """Run target(rank, world, port, q, *args) in `world` spawned processes; returns the
    per-rank results (each worker puts (rank, result))."""
    import torch.multiprocessing as mp
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(args)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=timeout)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [res[r] for r in range(world)]


def _init(rank, world, port):
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _pkgload
    return dist, _pkgload.load()


def callbacks_worker(rank, world, port, q):
    """Drive HostTransport through its C function pointers, as libpgmg calls them."""
    import numpy as np
    dist, pg = _init(rank, world, port)
    ht = pg.HostTransport()
    peers = [r for r in range(world) if r != rank]
    # two messages to every peer (posting order must be kept), sizes depend on the pair
    sends = []
    for r in peers:
        sends.append((r, np.full(10 + r, 16 * rank + r, dtype=np.uint8)))
        sends.append((r, np.arange(3 + rank, dtype=np.uint8)))
    recvs = []
    for r in peers:
        recvs.append((r, 10 + rank))
        recvs.append((r, 3 + r))
    rbufs = [np.zeros(n, dtype=np.uint8) for _, n in recvs]
    i_arr = lambda xs: (C.c_int * max(1, len(xs)))(*xs)
    u_arr = lambda xs: (C.c_ulonglong * max(1, len(xs)))(*xs)
    p_arr = lambda xs: (C.c_void_p * max(1, len(xs)))(*xs)
    rc = ht.struct.exchange(None, len(sends), i_arr([p for p, _ in sends]),
                            p_arr([a.ctypes.data for _, a in sends]), u_arr([a.size for _, a in sends]),
                            len(recvs), i_arr([p for p, _ in recvs]),
                            p_arr([b.ctypes.data for b in rbufs]), u_arr([n for _, n in recvs]))
    ok = rc == 0
    for k, r in enumerate(peers):
        ok &= bool((rbufs[2 * k] == 16 * r + rank).all()) and rbufs[2 * k].size == 10 + rank
        ok &= bool((rbufs[2 * k + 1] == np.arange(3 + r)).all())
    # rank-order sum: (0.0 + v_0) + v_1 + ... with values whose order matters in fp64
    v = np.array([1e16 if rank == 0 else 1.0, rank + 0.1], dtype=np.float64)
    rc2 = ht.struct.allreduce_sum_f64(None, v.ctypes.data_as(C.POINTER(C.c_double)), 2)
    want = np.zeros(2)
    for r in range(world):
        want += np.array([1e16 if r == 0 else 1.0, r + 0.1])
    ok &= rc2 == 0 and bool((v == want).all())
    u = np.array([rank + 1, 7, 1 if rank else 0], dtype=np.uint32)
    rc3 = ht.struct.allreduce_min_u32(None, u.ctypes.data_as(C.POINTER(C.c_uint)), 3)
    ok &= rc3 == 0 and u.tolist() == [1, 7, 0]
    q.put((rank, ok))
    dist.barrier()
    dist.destroy_process_group()


def solve_worker(rank, world, port, q, N, kind, cycles, cfg):
    """One rank of a row-strip solve over the host-staged transport, all ranks on GPU 0:
    the FNV-64 of the gathered phi (rank 0), sweeps and the transport's call count."""
    dist, pg = _init(rank, world, port)
    import torch  # noqa: F401
    ht = pg.HostTransport()
    cfg = dict(cfg)
    flags = 0
    if cfg.pop("exact", False):
        flags |= pg.PGMG_FLAG_EXACT_DIST
    with pg.Solver(N, transport=ht, device=0, flags=flags, **cfg) as s:
        s.set_problem()
        run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[kind]
        for _ in range(cycles):
            run(1)
        s.sync()
        h = s.solution_hash(0)
        sweeps, _ = s.stats()
        dinfo = s.dist_info()
    q.put((rank, {"hash": h, "sweeps": sweeps, "calls": ht.calls, "dist": list(dinfo)}))
    dist.barrier()
    dist.destroy_process_group()
