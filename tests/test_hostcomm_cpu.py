"""CPU, world 2 and 3 over gloo: the host-staged transport's callbacks (HostTransport,
PGMG_FLAG_HOST_TRANSPORT) called through their C function pointers, as libpgmg calls them:
point-to-point messages matched in posting order, the rank-order f64 sum every rank must
agree on, the u32 minimum of the speculative-validation flags."""
import pytest

from mp_workers import callbacks_worker, run_world


@pytest.mark.parametrize("world", [2, 3])
def test_host_transport_callbacks(world):
    assert all(run_world(callbacks_worker, world))
