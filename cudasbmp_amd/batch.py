"""Step-level entry points of the C ABI (include/sbmp/sbmp.h) over numpy
arrays: one stage of the KGMT iteration run alone on the GPU (or, for the expansion,
the same code on the host), so each stage can be checked against the CPU oracle.

    expand_batch  propagateG's per-child work (KGMT.cu:386-411): propagateAndCheck,
                  getR1 / getR2, the accept test
    insert_batch  exclusive_scan(GNew) + findInd + updateG (KGMT.cu:221-249, 540-593)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat


class _Dev:
    """A device copy of a numpy array (raw bytes), freed on close."""

    def __init__(self, host: np.ndarray):
        self.host = np.ascontiguousarray(host)
        p = ctypes.c_void_p()
        nat.call("sbmp_device_alloc", self.host.nbytes, ctypes.byref(p))
        self.ptr = p.value
        nat.call("sbmp_device_copy_to", ctypes.c_void_p(self.ptr), self.host.ctypes.data_as(ctypes.c_void_p),
                 self.host.nbytes)

    def get(self) -> np.ndarray:
        out = np.empty_like(self.host)
        nat.call("sbmp_device_copy_from", out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self.ptr), out.nbytes)
        return out

    def close(self):
        if self.ptr:
            nat.call("sbmp_device_free", ctypes.c_void_p(self.ptr))
            self.ptr = None


def expand_batch(parents, rng, obstacles, *, numDisc=10, agentLength=1.0, width=20.0, height=20.0, N=16, n=8,
                 agent="car", R1Score=None, R2Avail=None, device=True) -> dict:
    """parents (k, 7) float32, rng (k, 6) uint32 XORWOW states -> children (k, 7), valid, r1, r2,
    accept (R1Score / R2Avail given) and the advanced RNG states.  device=False runs the same
    code (the public headers) on the host."""
    par = np.ascontiguousarray(parents, dtype=np.float32).reshape(-1, 7)
    k = len(par)
    host = {"parents": par, "rng": np.ascontiguousarray(rng, dtype=np.uint32).reshape(-1, 6).copy(),
            "obstacles": np.ascontiguousarray(obstacles, dtype=np.float32).reshape(-1, 4),
            "children": np.zeros((k, 7), dtype=np.float32), "valid": np.zeros(k, dtype=np.uint8),
            "r1": np.zeros(k, dtype=np.int32), "r2": np.zeros(k, dtype=np.int32),
            "accept": np.zeros(k, dtype=np.uint8)}
    if R1Score is not None:
        host["R1Score"] = np.ascontiguousarray(R1Score, dtype=np.float32)
        host["R2Avail"] = np.ascontiguousarray(R2Avail, dtype=np.int32)
    a = nat.ExpandBatchArgs()
    a.count, a.obstaclesCount = k, len(host["obstacles"])
    a.agent = nat.SBMP_AGENT_POINT if agent == "point" else nat.SBMP_AGENT_CAR
    a.numDisc, a.agentLength, a.width, a.height, a.N, a.n = numDisc, agentLength, width, height, N, n
    devs = {}
    try:
        for name, arr in host.items():
            if device:
                devs[name] = _Dev(arr)
                setattr(a, name, devs[name].ptr)
            else:
                setattr(a, name, arr.ctypes.data)
        if device:
            nat.call("sbmp_expand_batch", ctypes.byref(a), None)
            out = {name: devs[name].get() for name in ("children", "valid", "r1", "r2", "accept", "rng")}
        else:
            nat.call("sbmp_expand_batch_host", ctypes.byref(a))
            out = {name: host[name] for name in ("children", "valid", "r1", "r2", "accept", "rng")}
    finally:
        for d in devs.values():
            d.close()
    return out


def insert_batch(gnew, unexplored, uParent, samples, parent, costs, treeSize, goal, goalThreshold,
                 fixGNewClear=False):
    """updateG over a batch on the GPU: returns (samples, parent, costs, gnew, A, goal row or -1)."""
    host = {"gnew": np.ascontiguousarray(gnew, dtype=np.uint8),
            "unexplored": np.ascontiguousarray(unexplored, dtype=np.float32),
            "uParent": np.ascontiguousarray(uParent, dtype=np.int32),
            "samples": np.ascontiguousarray(samples, dtype=np.float32),
            "parent": np.ascontiguousarray(parent, dtype=np.int32),
            "costs": np.ascontiguousarray(costs, dtype=np.float32),
            "inserted": np.zeros(1, dtype=np.int32), "goalIndex": np.zeros(1, dtype=np.int32)}
    a = nat.InsertBatchArgs()
    a.slots, a.treeSize, a.maxTreeSize = len(host["gnew"]), int(treeSize), len(host["parent"])
    a.goalX, a.goalY, a.goalThreshold, a.fixGNewClear = float(goal[0]), float(goal[1]), goalThreshold, int(fixGNewClear)
    devs = {}
    try:
        for name, arr in host.items():
            devs[name] = _Dev(arr)
            setattr(a, name, devs[name].ptr)
        nat.call("sbmp_insert_batch", ctypes.byref(a), None)
        r = {name: d.get() for name, d in devs.items()}
    finally:
        for d in devs.values():
            d.close()
    return r["samples"], r["parent"], r["costs"], r["gnew"], int(r["inserted"][0]), int(r["goalIndex"][0])
