"""GPU: the RCCL transport of the row-strip path, exercised for real on the one GPU of the
test box.  RCCL refuses two ranks on one device, so the strip tests run over the loopback
transport; this test drives the RCCL calls themselves (grouped ncclSend/ncclRecv,
ncclAllReduce sum/double and min/u32 on a stream) through a world-1 communicator
(pgmg_rccl_selftest, pgmg_comm.hip)."""
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
