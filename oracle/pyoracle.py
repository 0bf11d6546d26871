"""ctypes binding of oracle/_build/libkgmt_oracle.so — TEST INFRASTRUCTURE ONLY.

Mirrors the reference's KGMT interface (reference include/planners/KGMT.cuh:28-31:
ctor(width, height, N, n, numIterations, maxTreeSize, numDisc, agentLength,
goalThreshold), plan(initial, goal, obstacles, obstaclesCount)) with an explicit
curand seed, plus state accessors in the reference's array layouts.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libkgmt_oracle.so")
_lib = None


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_float), ("height", ctypes.c_float),
        ("N", ctypes.c_int), ("n", ctypes.c_int),
        ("numIterations", ctypes.c_int), ("maxTreeSize", ctypes.c_int), ("numDisc", ctypes.c_int),
        ("agentLength", ctypes.c_float), ("goalThreshold", ctypes.c_float),
        ("samplesPerIteration", ctypes.c_int), ("agent", ctypes.c_int),
        ("fixGNewClear", ctypes.c_int), ("threads", ctypes.c_int),
        ("nranks", ctypes.c_int), ("rank", ctypes.c_int), ("batchRule", ctypes.c_int),
    ]


class OracleRecord(ctypes.Structure):
    _fields_ = [("slot", ctypes.c_int32), ("sample", ctypes.c_float * 7), ("parent", ctypes.c_int32)]


RECORD_DTYPE = np.dtype([("slot", "<i4"), ("sample", "<f4", (7,)), ("parent", "<i4")])


class OracleIterLog(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("itr", "treeSizeBefore", "nG", "k", "nExp", "S", "A", "treeSizeAfter", "goalIdx")]


def build(quiet: bool = True) -> str:
    """Compile the oracle with its Makefile (g++, no GPU needed)."""
    out = subprocess.run(["make", "-C", _HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i, f, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64
        P = ctypes.POINTER
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [P(OracleParams)]
        L.oracle_destroy.argtypes = [vp]
        for name in ("oracle_begin", "oracle_plan"):
            getattr(L, name).argtypes = [vp, P(f), P(f), P(f), i, u64]
            getattr(L, name).restype = i
        for name in ("oracle_step", "oracle_expand_local", "oracle_delta_size", "oracle_num_slots"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = i
        L.oracle_local_records.argtypes = [vp, vp, i]
        L.oracle_local_deltas.argtypes = [vp, vp]
        L.oracle_finish.argtypes = [vp, vp, i, vp]
        L.oracle_finish.restype = i
        L.oracle_info.argtypes = [vp, P(i), P(i), P(i), P(f), P(i)]
        L.oracle_tree.argtypes = [vp, vp, vp, vp]
        L.oracle_unexplored.argtypes = [vp, vp, vp]
        L.oracle_flags.argtypes = [vp, vp, vp]
        L.oracle_regions.argtypes = [vp] + [vp] * 8
        L.oracle_rng.argtypes = [vp, vp]
        L.oracle_iter_logs.argtypes = [vp, vp, i]
        L.oracle_iter_logs.restype = i
        L.oracle_samples_generated.argtypes = [vp]
        L.oracle_samples_generated.restype = ctypes.c_longlong
        L.oracle_xorwow_init.argtypes = [u64, u64, i, vp]
        L.oracle_xorwow_draw.argtypes = [vp, i, vp]
        L.oracle_replay.argtypes = [P(OracleParams), vp, i, vp, vp, i, vp, vp]
        L.oracle_sincosf.argtypes = [vp, i, vp, vp]
        L.oracle_expand_batch.argtypes = [P(OracleParams), vp, i, vp, vp, i, vp, vp, vp, vp, vp, vp, vp]
        L.oracle_random_tree.argtypes = [i, vp, i, i, i, vp]
        L.oracle_tanf.argtypes = [vp, i, vp]
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class PlannerConfig:
    width: float = 20.0
    height: float = 20.0
    N: int = 16
    n: int = 8
    numIterations: int = 100
    maxTreeSize: int = 30000
    numDisc: int = 10
    agentLength: float = 1.0
    goalThreshold: float = 0.5
    samplesPerIteration: int = 0
    agent: int = 0
    fixGNewClear: int = 0
    batchRule: int = 0


class Oracle:
    """One CPU planner instance (reference KGMT semantics + D1-D13)."""

    def __init__(self, cfg: PlannerConfig, threads: int = 1, nranks: int = 1, rank: int = 0):
        self.cfg = cfg
        p = OracleParams(cfg.width, cfg.height, cfg.N, cfg.n, cfg.numIterations, cfg.maxTreeSize,
                         cfg.numDisc, cfg.agentLength, cfg.goalThreshold, cfg.samplesPerIteration,
                         cfg.agent, cfg.fixGNewClear, threads, nranks, rank, cfg.batchRule)
        self._h = lib().oracle_create(ctypes.byref(p))
        if not self._h:
            raise ValueError("oracle_create rejected the parameters")
        self.M = cfg.maxTreeSize
        self.nR1 = cfg.N * cfg.N
        self.nR2 = self.nR1 * cfg.n * cfg.n

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_destroy(self._h)
            self._h = None

    @staticmethod
    def _arr7(v):
        a = np.zeros(7, dtype=np.float32)
        v = np.asarray(v, dtype=np.float32).ravel()
        a[: len(v)] = v
        return a

    def begin(self, initial, goal, obstacles, seed: int):
        self._init = self._arr7(initial)
        self._goal = self._arr7(goal)
        self._obs = np.ascontiguousarray(obstacles, dtype=np.float32).ravel()
        FP = ctypes.POINTER(ctypes.c_float)
        lib().oracle_begin(self._h, self._init.ctypes.data_as(FP), self._goal.ctypes.data_as(FP),
                           self._obs.ctypes.data_as(FP), len(self._obs) // 4, seed)

    def step(self) -> bool:
        return bool(lib().oracle_step(self._h))

    def plan(self, initial, goal, obstacles, seed: int) -> int:
        self.begin(initial, goal, obstacles, seed)
        n = 0
        while self.step():
            n += 1
        return n

    # sharded protocol
    def expand_local(self) -> int:
        return lib().oracle_expand_local(self._h)

    def local_records(self) -> np.ndarray:
        cap = max(1, self.M)
        out = np.zeros(cap, dtype=RECORD_DTYPE)
        n = lib().oracle_local_records(self._h, _fp(out), cap)
        return out[:n].copy()

    def local_deltas(self) -> np.ndarray:
        out = np.zeros(lib().oracle_delta_size(self._h), dtype=np.int32)
        lib().oracle_local_deltas(self._h, _fp(out))
        return out

    def finish(self, records: np.ndarray, summed_deltas: np.ndarray) -> int:
        records = np.ascontiguousarray(records, dtype=RECORD_DTYPE)
        summed_deltas = np.ascontiguousarray(summed_deltas, dtype=np.int32)
        return lib().oracle_finish(self._h, _fp(records), len(records), _fp(summed_deltas))

    # accessors
    def info(self) -> dict:
        itr, ts, gi, term = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        c = ctypes.c_float()
        lib().oracle_info(self._h, ctypes.byref(itr), ctypes.byref(ts), ctypes.byref(gi), ctypes.byref(c),
                          ctypes.byref(term))
        return {"iterations": itr.value, "treeSize": ts.value, "goalIdx": gi.value,
                "costToGoal": c.value, "terminated": bool(term.value),
                "samples": int(lib().oracle_samples_generated(self._h))}

    def tree(self):
        s = np.zeros((self.M, 7), dtype=np.float32)
        p = np.zeros(self.M, dtype=np.int32)
        c = np.zeros(self.M, dtype=np.float32)
        lib().oracle_tree(self._h, _fp(s), _fp(p), _fp(c))
        return s, p, c

    def unexplored(self):
        s = np.zeros((self.M, 7), dtype=np.float32)
        p = np.zeros(self.M, dtype=np.int32)
        lib().oracle_unexplored(self._h, _fp(s), _fp(p))
        return s, p

    def flags(self):
        g = np.zeros(self.M, dtype=np.uint8)
        gn = np.zeros(self.M, dtype=np.uint8)
        lib().oracle_flags(self._h, _fp(g), _fp(gn))
        return g, gn

    def regions(self) -> dict:
        r = {k: np.zeros(self.nR1, dtype=np.int32) for k in ("R1", "R1Avail", "R1Valid", "R1Invalid")}
        r["R1Score"] = np.zeros(self.nR1, dtype=np.float32)
        for k in ("R2Avail", "R2Valid", "R2Invalid"):
            r[k] = np.zeros(self.nR2, dtype=np.int32)
        lib().oracle_regions(self._h, *[_fp(r[k]) for k in ("R1", "R1Avail", "R1Valid", "R1Invalid", "R1Score",
                                                             "R2Avail", "R2Valid", "R2Invalid")])
        return r

    def rng(self) -> np.ndarray:
        n = lib().oracle_num_slots(self._h)
        out = np.zeros((n, 6), dtype=np.uint32)
        lib().oracle_rng(self._h, _fp(out))
        return out

    def iter_logs(self) -> np.ndarray:
        cap = 1 << 16
        arr = (OracleIterLog * cap)()
        n = lib().oracle_iter_logs(self._h, ctypes.cast(arr, ctypes.c_void_p), cap)
        names = [f[0] for f in OracleIterLog._fields_]
        return np.array([[getattr(arr[i], k) for k in names] for i in range(n)], dtype=np.int64).reshape(-1, len(names))


def replay(cfg: PlannerConfig, obstacles, parents: np.ndarray, controls: np.ndarray, threads: int = 8):
    """Invariant I1: re-propagate parents (n,4) with controls (n,3) -> (states (n,4), valid (n,))."""
    p = OracleParams(cfg.width, cfg.height, cfg.N, cfg.n, cfg.numIterations, cfg.maxTreeSize, cfg.numDisc,
                     cfg.agentLength, cfg.goalThreshold, cfg.samplesPerIteration, cfg.agent, cfg.fixGNewClear,
                     threads, 1, 0, cfg.batchRule)
    obs = np.ascontiguousarray(obstacles, dtype=np.float32).ravel()
    parents = np.ascontiguousarray(parents, dtype=np.float32)
    controls = np.ascontiguousarray(controls, dtype=np.float32)
    n = len(parents)
    out = np.zeros((n, 4), dtype=np.float32)
    valid = np.zeros(n, dtype=np.uint8)
    lib().oracle_replay(ctypes.byref(p), _fp(obs), len(obs) // 4, _fp(parents), _fp(controls), n, _fp(out),
                        _fp(valid))
    return out, valid.astype(bool)


def expand_batch(cfg: PlannerConfig, obstacles, parents: np.ndarray, rng: np.ndarray, R1Score=None, R2Avail=None,
                 threads: int = 8) -> dict:
    """propagateG's per-child work over a batch (KGMT.cu:386-411): parents (n, 7), rng (n, 6)
    uint32 XORWOW states -> children (n, 7), valid, r1, r2, accept (R1Score / R2Avail given)
    and the advanced RNG states.  The checker of sbmp_expand_batch."""
    p = OracleParams(cfg.width, cfg.height, cfg.N, cfg.n, cfg.numIterations, cfg.maxTreeSize, cfg.numDisc,
                     cfg.agentLength, cfg.goalThreshold, cfg.samplesPerIteration, cfg.agent, cfg.fixGNewClear,
                     threads, 1, 0, cfg.batchRule)
    obs = np.ascontiguousarray(obstacles, dtype=np.float32).ravel()
    par = np.ascontiguousarray(parents, dtype=np.float32)
    st = np.ascontiguousarray(rng, dtype=np.uint32).copy()
    n = len(par)
    out = {"children": np.zeros((n, 7), dtype=np.float32), "valid": np.zeros(n, dtype=np.uint8),
           "r1": np.zeros(n, dtype=np.int32), "r2": np.zeros(n, dtype=np.int32),
           "accept": np.zeros(n, dtype=np.uint8)}
    sc = None if R1Score is None else np.ascontiguousarray(R1Score, dtype=np.float32)
    av = None if R2Avail is None else np.ascontiguousarray(R2Avail, dtype=np.int32)
    lib().oracle_expand_batch(ctypes.byref(p), _fp(obs), len(obs) // 4, _fp(par), _fp(st), n,
                              None if sc is None else _fp(sc), None if av is None else _fp(av),
                              _fp(out["children"]), _fp(out["valid"]), _fp(out["r1"]), _fp(out["r2"]),
                              _fp(out["accept"]))
    out["rng"] = st
    return out


def insert_batch(gnew: np.ndarray, unexplored: np.ndarray, uParent: np.ndarray, samples: np.ndarray,
                 parent: np.ndarray, costs: np.ndarray, treeSize: int, goal, goalThreshold: float,
                 fixGNewClear: bool = False):
    """updateG over a batch (KGMT.cu:221-249 exclusive_scan(GNew) + findInd + updateG, 540-593),
    in place on copies: the accepted slots, in slot order, become rows treeSize + j with
    parent uParent, cost = cost[parent] + duration (getCost, KGMT.cu:631-633); only
    min(A, 32 floor(M/32)) rows are written (the updateG grid, KGMT.cu:231) and none past M
    (D13); GNew[0 .. 32 min(A, M/32)) is cleared (D6; everything with fixGNewClear).
    Returns (samples, parent, costs, gnew, A, lowest new row in the goal region or -1)."""
    samples, parent, costs, gnew = samples.copy(), parent.copy(), costs.copy(), gnew.copy()
    M = len(parent)
    idx = np.nonzero(gnew)[0]
    A = len(idx)
    grid = min(A, M // 32)
    nIns = min(A, 32 * grid)
    goal_row = -1
    for j in range(nIns):
        dst = treeSize + j
        if dst >= M:
            break
        s = idx[j]
        parent[dst] = uParent[s]
        samples[dst] = unexplored[s]
        costs[dst] = np.float32(costs[uParent[s]] + unexplored[s, 6])
        dx = np.float32(unexplored[s, 0] - np.float32(goal[0]))
        dy = np.float32(unexplored[s, 1] - np.float32(goal[1]))
        if goal_row < 0 and np.sqrt(np.float32(dx * dx + dy * dy), dtype=np.float32) < np.float32(goalThreshold):
            goal_row = dst
    if fixGNewClear:
        gnew[:] = 0
    else:
        gnew[:32 * grid] = 0
    return samples, parent, costs, gnew, A, goal_row


def random_tree(kind: str, root, rows: int, blocks: int, tpb: int) -> np.ndarray:
    """Legacy generators: kind 'naive' (NaivePlanner.cu) or 'costprop'
    (CostPropPlanner.cu) -> (rows, blocks * tpb, 7) samples."""
    r = np.ascontiguousarray(np.asarray(root, dtype=np.float32)[:7])
    out = np.zeros((rows, blocks * tpb, 7), dtype=np.float32)
    lib().oracle_random_tree(0 if kind == "naive" else 1, _fp(r), rows, blocks, tpb, _fp(out))
    return out


def xorwow_init(seed: int, subsequence: int, seeding: str = "curand") -> np.ndarray:
    st = np.zeros(6, dtype=np.uint32)
    lib().oracle_xorwow_init(seed, subsequence, 0 if seeding == "curand" else 1, _fp(st))
    return st


def xorwow_draw(state: np.ndarray, count: int) -> np.ndarray:
    out = np.zeros(count, dtype=np.uint32)
    lib().oracle_xorwow_draw(_fp(state), count, _fp(out))
    return out


def sincosf(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    lib().oracle_sincosf(_fp(x), len(x), _fp(s), _fp(c))
    return s, c


def tanf(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    t = np.zeros_like(x)
    lib().oracle_tanf(_fp(x), len(x), _fp(t))
    return t
