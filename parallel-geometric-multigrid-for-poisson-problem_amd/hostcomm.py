"""HostTransport: pgmg_host_transport (include/pgmg.h) over a torch.distributed group.

The row-strip decomposition normally moves its halos and gathered rows with RCCL, one
process per GPU.  With PGMG_FLAG_HOST_TRANSPORT the library stages every message through
host memory and calls back into the functions of this object, which move them with
torch.distributed point-to-point calls and all_gather on the caller's group (gloo on the
host).  Ranks may then share one GPU — the multi-process path can be run end to end on a
one-GPU box, bitwise against one GPU.  It is plumbing for correctness, not a fast path.

Semantics (the RCCL path's): one exchange() per group of messages, messages between two
ranks matched in posting order; allreduce sums in rank order (0.0 + v_0 + v_1 + ...), so
every rank takes the same early-exit decisions as the in-process loopback transport.
"""
import ctypes as C
import sys
import traceback

import numpy as np

from ._capi import HT_EXCHANGE, HT_MIN_U32, HT_SUM_F64, PgmgHostTransport


class HostTransport:
    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self._torch = torch
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.calls = 0
        # keep the ctypes callback objects alive as long as this object
        self._cbs = (HT_EXCHANGE(self._exchange), HT_SUM_F64(self._sum_f64),
                     HT_MIN_U32(self._min_u32))
        self.struct = PgmgHostTransport(None, *self._cbs)

    def _peer(self, r):
        """rank within the group -> global rank (what torch.distributed's p2p calls take)"""
        if self.group is None:
            return r
        return self._dist.get_global_rank(self.group, r)

    def exchange_arrays(self, sends, recv_specs):
        """sends: [(peer, uint8 array)], recv_specs: [(peer, nbytes)] -> [uint8 array]"""
        torch, dist = self._torch, self._dist
        reqs, outs = [], []
        for peer, a in sends:
            if a.size:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a)), self._peer(peer),
                                       group=self.group))
        for peer, n in recv_specs:
            t = torch.empty(n, dtype=torch.uint8)
            if n:
                reqs.append(dist.irecv(t, self._peer(peer), group=self.group))
            outs.append(t)
        for q in reqs:
            q.wait()
        return [t.numpy() for t in outs]

    def allreduce_sum(self, v):
        """rank-order sum of a float64 vector over the group"""
        torch = self._torch
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self._dist.all_gather(parts, t, group=self.group)
        tot = np.zeros(t.numel(), dtype=np.float64)
        for p in parts:   # 0.0 + v_0 + v_1 + ...: the loopback transport's order
            tot += p.numpy()
        return tot

    def allreduce_min(self, v):
        torch = self._torch
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64))
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self._dist.all_gather(parts, t, group=self.group)
        return np.minimum.reduce([p.numpy() for p in parts])

    # ---- the C callbacks -------------------------------------------------------------
    def _exchange(self, user, nsend, speer, sbuf, sbytes, nrecv, rpeer, rbuf, rbytes):
        try:
            self.calls += 1
            sends = []
            for i in range(nsend):
                n = int(sbytes[i])
                a = np.empty(n, dtype=np.uint8)
                if n:
                    C.memmove(a.ctypes.data, sbuf[i], n)
                sends.append((int(speer[i]), a))
            outs = self.exchange_arrays(sends, [(int(rpeer[i]), int(rbytes[i])) for i in range(nrecv)])
            for i, a in enumerate(outs):
                if a.size:
                    C.memmove(rbuf[i], a.ctypes.data, a.size)
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1

    def _sum_f64(self, user, v, n):
        try:
            a = np.ctypeslib.as_array(v, shape=(n,))
            a[:] = self.allreduce_sum(a.copy())
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1

    def _min_u32(self, user, v, n):
        try:
            a = np.ctypeslib.as_array(v, shape=(n,))
            a[:] = self.allreduce_min(a.astype(np.int64)).astype(np.uint32)
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1
