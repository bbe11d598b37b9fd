"""GPU: the RCCL transport of the row-strip path, exercised for real on the one GPU of the
test box.  RCCL refuses two ranks on one device, so the strip tests run over the loopback
transport; this test drives the RCCL calls themselves (grouped ncclSend/ncclRecv,
ncclAllReduce sum/double and min/u32 on a stream) through a world-1 communicator, and the
early finest-level halo's pattern: a communicator split off it (ncclCommSplit) exchanging
on a second stream that waits for the first, while the first runs its reductions, both
polled by one wait (pgmg_rccl_selftest, pgmg_comm.hip)."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_transport_selftest(pgmg):
    import torch
    assert torch.cuda.is_available()
    uid = (C.c_ubyte * 128)(*pgmg.unique_id())
    lib = pgmg.load()
    rc = lib.pgmg_rccl_selftest(C.cast(uid, C.c_void_p), 0)
    assert rc == 0, lib.pgmg_last_error()


@pytest.mark.parametrize("world,rank", [(2, 0), (2, 1), (8, 3)])
def test_solo_rank_runs(pgmg, world, rank):
    """PGMG_FLAG_SOLO (measurement mode of scripts/strip_probe.py): one rank of a world-W
    strip decomposition on one GPU with the null transport runs V, W and F cycles (the
    values are meaningless; the test pins that the mode works and plans the strips)."""
    with pgmg.Solver(1025, rank=rank, world=world, flags=pgmg.PGMG_FLAG_SOLO, gather_n=65) as s:
        s.set_problem()
        s.vcycle(2)
        s.wcycle(1)
        s.fcycle(1)
        s.sync()
        lo, hi, nd = pgmg.plan_strips(1025, world, rank, 65, 65)
        assert nd > 0 and hi > lo
