"""Host-staged transport over a torch.distributed process group.

lssp_amd_comm_init_host (include/lssp_amd.h) lets the caller carry the
multi-rank protocol's collectives instead of RCCL: an all-gather of a few
bytes per rank (dot partials, setup counts) and one grouped point-to-point
round per halo exchange.  This module implements those two hooks with
torch.distributed on CPU tensors (gloo), so the full distributed path --
partition, halo plan, pack kernel, rank-order dot sums, block-Jacobi ILU --
runs with several ranks on ONE GPU, which RCCL refuses ("Duplicate GPU").
Production multi-GPU runs use RCCL (Device.comm_init).
"""
from __future__ import annotations

import ctypes
import traceback

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def _bytes_at(ptr, n: int) -> np.ndarray:
    return np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(ptr))[:n]


class GlooTransport:
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.struct = _lib.HostTransport(None, _lib.ALLGATHER_FN(self._allgather),
                                         _lib.SENDRECV_FN(self._sendrecv))

    def _allgather(self, _user, send, recv, nbytes):
        try:
            src = torch.from_numpy(_bytes_at(send, nbytes).copy())
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
            dist.all_gather(outs, src, group=self.group)
            dst = _bytes_at(recv, nbytes * self.world)
            for q, o in enumerate(outs):
                dst[q * nbytes:(q + 1) * nbytes] = o.numpy()
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def _sendrecv(self, _user, ns, sp, sb, sl, nr, rp, rb, rl):
        try:
            ops, bufs = [], []
            for i in range(ns):
                t = torch.from_numpy(_bytes_at(sb[i], sl[i]).copy())
                ops.append(dist.P2POp(dist.isend, t, sp[i], group=self.group))
            for i in range(nr):
                t = torch.empty(rl[i], dtype=torch.uint8)
                bufs.append((t, rb[i], rl[i]))
                ops.append(dist.P2POp(dist.irecv, t, rp[i], group=self.group))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            for t, ptr, n in bufs:
                _bytes_at(ptr, n)[:] = t.numpy()
            return 0
        except Exception:
            traceback.print_exc()
            return 1
