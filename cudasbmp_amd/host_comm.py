"""Host collectives for the sharded planner (sbmp_kgmt_create_sharded_host) over
torch.distributed -- e.g. the gloo backend for several processes on one GPU, where
RCCL cannot put two ranks on one device.  The planner synchronises its stream,
copies the fused exchange buffer to host memory and calls these callbacks; the
record buffers themselves are still read over HIP IPC by the kernels.
"""
from __future__ import annotations

import ctypes
import sys

import numpy as np

from . import _native as nat


class TorchCollectives:
    """sbmp_host_collectives backed by an initialised torch.distributed process group."""

    def __init__(self, dist, group=None):
        import torch
        self._dist, self._group, self._torch = dist, group, torch

        def _guard(fn):
            def run(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:   # a C callback must not raise
                    print(f"host collective failed: {e!r}", file=sys.stderr, flush=True)
                    return 1
            return run

        def _allreduce(dtype, ctype):
            def fn(_ctx, send, recv, count):
                src = np.ctypeslib.as_array((ctype * count).from_address(send)).view(dtype)
                t = torch.from_numpy(src.copy())
                dist.all_reduce(t, group=group)   # integer sums wrap like the device counters
                np.ctypeslib.as_array((ctype * count).from_address(recv)).view(dtype)[:] = t.numpy()
            return fn

        def allgather(_ctx, send, nbytes, recv):
            src = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(send))
            t = torch.from_numpy(src.copy())
            out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
            dist.all_gather(out, t, group=group)
            dst = np.ctypeslib.as_array((ctypes.c_uint8 * (nbytes * len(out))).from_address(recv))
            dst[:] = np.concatenate([o.numpy() for o in out])

        self._fns = (nat.ALLREDUCE_FN(_guard(_allreduce(np.int64, ctypes.c_uint64))),
                     nat.ALLREDUCE_FN(_guard(_allreduce(np.int32, ctypes.c_int32))),
                     nat.ALLGATHER_FN(_guard(allgather)))
        self.struct = nat.HostCollectives(None, *self._fns)
