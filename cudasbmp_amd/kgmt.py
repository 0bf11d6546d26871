"""Python mirror of the reference planner interface, backed by libsbmp.so.

Reference: class KGMT (include/planners/KGMT.cuh:23-109)
    KGMT(float width, float height, int N, int n, int numIterations, int maxTreeSize,
         int numDisc, float agentLength, float goalThreshold)
    void plan(float* initial, float* goal, float* d_obstacles, int obstaclesCount)
    public fields treeSize_, costToGoal_, numIterations_, maxTreeSize_, numDisc_, width_,
                  height_, agentLength_, goalThreshold_, N_, n_, R1Size_, R2Size_
The reference seeds curand with time(NULL) inside plan() (KGMT.cu:111); here the
seed is an optional keyword (default: time(NULL) converted int -> unsigned long
long exactly as the reference's initCurandStates(..., int seed) call does).
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np

from . import _native as nat

AGENTS = {"car": nat.SBMP_AGENT_CAR, "point": nat.SBMP_AGENT_POINT}
BATCH_RULES = {"reference": nat.SBMP_BATCH_REFERENCE, "fill": nat.SBMP_BATCH_FILL}


def reference_seed_from_time(t: Optional[float] = None) -> int:
    """time(NULL) -> int -> unsigned long long (sign-extended), as KGMT.cu:111 + curand_init."""
    v = ctypes.c_int(int(time.time() if t is None else t)).value
    return v & 0xFFFFFFFFFFFFFFFF


class DeviceBuffer:
    """A float32 device array allocated through the ABI (demos/main.cu:60-61 cudaMalloc+cudaMemcpy)."""

    def __init__(self, host: np.ndarray):
        host = np.ascontiguousarray(host, dtype=np.float32).ravel()
        p = ctypes.c_void_p()
        nat.call("sbmp_device_upload_f32", host.ctypes.data_as(ctypes.c_void_p), host.size, ctypes.byref(p))
        self.ptr = p.value or 0
        self.count = host.size

    def free(self):
        if self.ptr:
            nat.call("sbmp_device_free", ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_ptr(obj) -> int:
    """Device address of a DeviceBuffer, a torch tensor on the GPU, or a raw int."""
    if obj is None:
        return 0
    if isinstance(obj, DeviceBuffer):
        return obj.ptr
    if isinstance(obj, int):
        return obj
    if hasattr(obj, "data_ptr"):
        if hasattr(obj, "is_cuda") and not obj.is_cuda:
            raise ValueError("d_obstacles must live in device memory")
        return obj.data_ptr()
    raise TypeError(f"cannot take a device pointer of {type(obj)!r}")


def random_tree(kind: str, root, rows: int = 0, blocks: int = 0, threads_per_block: int = 0, device: int = 0):
    """Legacy random-tree generators of the reference's Planner interface:
    kind 'naive' (NaivePlanner.cu) or 'costprop' (CostPropPlanner.cu); sizes <= 0 take the
    reference's.  Returns (samples (rows, blocks * threads_per_block, 7) float32, kernel ms)."""
    naive = kind == "naive"
    if kind not in ("naive", "costprop"):
        raise ValueError("kind must be 'naive' or 'costprop'")
    rows = rows if rows > 0 else (10 if naive else 1)
    blocks = blocks if blocks > 0 else (32 if naive else 512)
    tpb = threads_per_block if threads_per_block > 0 else (32 if naive else 1024)
    r = np.zeros(7, dtype=np.float32)
    r[: len(root)] = np.asarray(root, dtype=np.float32)[:7]
    out = np.zeros((rows, blocks * tpb, 7), dtype=np.float32)
    ms = ctypes.c_float()
    nat.call("sbmp_random_tree", device, 0 if naive else 1, r.ctypes.data_as(ctypes.c_void_p), rows, blocks, tpb,
             out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(ms))
    return out, ms.value


def read_obstacles_csv(path: str, workspace_dim: int = 2) -> np.ndarray:
    """readObstaclesFromCSV (reference src/helper/helper.cu:11-34) through the ABI; (count, 4) float32."""
    n = ctypes.c_int()
    nat.call("sbmp_read_obstacles_csv", path.encode(), workspace_dim, None, 0, ctypes.byref(n))
    cap = max(1, n.value * 2 * workspace_dim + 2 * workspace_dim)
    buf = np.zeros(cap, dtype=np.float32)
    nat.call("sbmp_read_obstacles_csv", path.encode(), workspace_dim, buf.ctypes.data_as(ctypes.c_void_p), cap,
             ctypes.byref(n))
    return buf[: n.value * 2 * workspace_dim].reshape(n.value, 2 * workspace_dim).copy()


def device_count() -> int:
    n = ctypes.c_int()
    nat.call("sbmp_device_count", ctypes.byref(n))
    return n.value


def hbm_copy_bandwidth(nbytes: int = 4 << 30, reps: int = 5) -> float:
    """Measured HBM copy bandwidth of the current device in GB/s (sbmp_hbm_copy_bandwidth)."""
    g = ctypes.c_double()
    nat.call("sbmp_hbm_copy_bandwidth", ctypes.c_size_t(nbytes), reps, ctypes.byref(g))
    return g.value


def _vec7(v) -> np.ndarray:
    a = np.zeros(7, dtype=np.float32)
    v = np.asarray(v, dtype=np.float32).ravel()
    a[: len(v)] = v
    return a


class KGMT:
    """MI355X KGMT planner with the reference's constructor and plan() signature."""

    def __init__(self, width: float, height: float, N: int, n: int, numIterations: int, maxTreeSize: int,
                 numDisc: int, agentLength: float, goalThreshold: float, *, samplesPerIteration: int = 0,
                 agent: str = "car", fixGNewClear: bool = False, device: int = 0, profileKernels: bool = False,
                 batchRule: str = "reference", _sharded=None, _local_group: int = 0, _host_sharded=None):
        p = nat.KgmtParams()
        nat.call("sbmp_kgmt_default_params", ctypes.byref(p))
        p.width, p.height, p.N, p.n = width, height, N, n
        p.numIterations, p.maxTreeSize, p.numDisc = numIterations, maxTreeSize, numDisc
        p.agentLength, p.goalThreshold = agentLength, goalThreshold
        p.samplesPerIteration = samplesPerIteration
        p.agent = AGENTS[agent]
        p.fixGNewClear = int(bool(fixGNewClear))
        p.device = device
        p.profileKernels = int(bool(profileKernels))
        p.batchRule = BATCH_RULES[batchRule]
        self._params = p
        h = ctypes.c_void_p()
        self._coll = None
        if _local_group:   # sharded data flow with virtual ranks on one device (tests)
            nat.call("sbmp_kgmt_create_local_group", ctypes.byref(p), int(_local_group), ctypes.byref(h))
        elif _host_sharded is not None:   # sharded, collectives by host callbacks (cudasbmp_amd.host_comm)
            coll, nranks, rank = _host_sharded
            self._coll = coll   # the callbacks must outlive the planner
            nat.call("sbmp_kgmt_create_sharded_host", ctypes.byref(p), ctypes.byref(coll.struct), nranks, rank,
                     ctypes.byref(h))
        elif _sharded is None:
            nat.call("sbmp_kgmt_create", ctypes.byref(p), ctypes.byref(h))
        else:
            uid, nranks, rank = _sharded
            idbuf = (ctypes.c_uint8 * nat.SBMP_COMM_ID_BYTES).from_buffer_copy(bytes(uid))
            nat.call("sbmp_kgmt_create_sharded", ctypes.byref(p), idbuf, nranks, rank, ctypes.byref(h))
        self._h = h
        # reference public fields (KGMT.cuh:34-43, 103-106)
        self.width_, self.height_, self.N_, self.n_ = float(width), float(height), N, n
        self.numIterations_, self.maxTreeSize_, self.numDisc_ = numIterations, maxTreeSize, numDisc
        self.agentLength_, self.goalThreshold_ = float(agentLength), float(goalThreshold)
        self.R1Size_ = float(np.float32(width) / np.float32(N))
        self.R2Size_ = float(np.float32(width) / np.float32(n * N))
        self.treeSize_ = 0
        self.costToGoal_ = 0.0
        self.last_result: Optional[nat.PlanResult] = None
        self._obs_keepalive = None

    @classmethod
    def from_params(cls, **kw) -> "KGMT":
        base = dict(width=20.0, height=20.0, N=16, n=8, numIterations=100, maxTreeSize=30000, numDisc=10,
                    agentLength=1.0, goalThreshold=0.5)
        base.update(kw)
        return cls(**base)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            nat.call("sbmp_kgmt_destroy", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def M(self) -> int:
        return self.maxTreeSize_

    # ---------------------------------------------------------------- planning
    def plan(self, initial, goal, d_obstacles, obstaclesCount: int, seed: Optional[int] = None) -> nat.PlanResult:
        """KGMT::plan (reference KGMT.cu:80-317); blocking."""
        seed = reference_seed_from_time() if seed is None else seed
        i, g = _vec7(initial), _vec7(goal)
        r = nat.PlanResult()
        self._obs_keepalive = d_obstacles
        nat.call("sbmp_kgmt_plan", self._h, i.ctypes.data_as(ctypes.c_void_p), g.ctypes.data_as(ctypes.c_void_p),
                 ctypes.c_void_p(device_ptr(d_obstacles)), obstaclesCount, seed, ctypes.byref(r))
        self._absorb(r)
        return r

    def begin(self, initial, goal, d_obstacles, obstaclesCount: int, seed: int) -> None:
        i, g = _vec7(initial), _vec7(goal)
        self._obs_keepalive = d_obstacles
        nat.call("sbmp_kgmt_begin", self._h, i.ctypes.data_as(ctypes.c_void_p), g.ctypes.data_as(ctypes.c_void_p),
                 ctypes.c_void_p(device_ptr(d_obstacles)), obstaclesCount, seed)

    def step(self, iterations: int = 1) -> bool:
        """Run up to `iterations` more loop iterations; False once the loop has ended."""
        a = ctypes.c_int()
        nat.call("sbmp_kgmt_step", self._h, iterations, ctypes.byref(a))
        return bool(a.value)

    def enqueue(self, iterations: int) -> None:
        nat.call("sbmp_kgmt_enqueue", self._h, iterations)

    def sync(self) -> None:
        nat.call("sbmp_kgmt_sync", self._h)

    def fold(self) -> None:
        """Enqueue the R2Valid / R2Invalid fold of every iteration enqueued so far (no wait)."""
        nat.call("sbmp_kgmt_fold", self._h)

    def result(self) -> nat.PlanResult:
        r = nat.PlanResult()
        nat.call("sbmp_kgmt_result", self._h, ctypes.byref(r))
        self._absorb(r)
        return r

    def _absorb(self, r: nat.PlanResult) -> None:
        self.treeSize_ = r.treeSize
        self.costToGoal_ = r.costToGoal
        self.last_result = r

    def stream(self) -> int:
        s = ctypes.c_void_p()
        nat.call("sbmp_kgmt_stream", self._h, ctypes.byref(s))
        return s.value or 0

    # ---------------------------------------------------------------- state export
    def tree(self):
        M = self.M
        s = np.zeros((M, 7), dtype=np.float32)
        p = np.zeros(M, dtype=np.int32)
        c = np.zeros(M, dtype=np.float32)
        nat.call("sbmp_kgmt_copy_tree", self._h, s.ctypes.data_as(ctypes.c_void_p),
                 p.ctypes.data_as(ctypes.c_void_p), c.ctypes.data_as(ctypes.c_void_p), M)
        return s, p, c

    def solution_path(self, node: int = -1):
        """Rows root .. node (default: the solution node) with their samples (n, 7) and
        costs; empty arrays when there is no solution."""
        n = ctypes.c_int()
        nat.call("sbmp_kgmt_solution_path", self._h, int(node), None, None, None, 0, ctypes.byref(n))
        rows = np.zeros(n.value, dtype=np.int32)
        s = np.zeros((n.value, 7), dtype=np.float32)
        c = np.zeros(n.value, dtype=np.float32)
        if n.value:
            nat.call("sbmp_kgmt_solution_path", self._h, int(node), rows.ctypes.data_as(ctypes.c_void_p),
                     s.ctypes.data_as(ctypes.c_void_p), c.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n))
        return rows, s, c

    def unexplored(self):
        M = self.M
        s = np.zeros((M, 7), dtype=np.float32)
        p = np.zeros(M, dtype=np.int32)
        nat.call("sbmp_kgmt_copy_unexplored", self._h, s.ctypes.data_as(ctypes.c_void_p),
                 p.ctypes.data_as(ctypes.c_void_p), M)
        return s, p

    def flags(self):
        M = self.M
        g = np.zeros(M, dtype=np.uint8)
        gn = np.zeros(M, dtype=np.uint8)
        nat.call("sbmp_kgmt_copy_flags", self._h, g.ctypes.data_as(ctypes.c_void_p),
                 gn.ctypes.data_as(ctypes.c_void_p), M)
        return g, gn

    def regions(self) -> dict:
        n1 = self.N_ * self.N_
        n2 = n1 * self.n_ * self.n_
        r = {k: np.zeros(n1, dtype=np.int32) for k in ("R1", "R1Avail", "R1Valid", "R1Invalid")}
        r["R1Score"] = np.zeros(n1, dtype=np.float32)
        for k in ("R2Avail", "R2Valid", "R2Invalid"):
            r[k] = np.zeros(n2, dtype=np.int32)
        order = ("R1", "R1Avail", "R1Valid", "R1Invalid", "R1Score", "R2Avail", "R2Valid", "R2Invalid")
        nat.call("sbmp_kgmt_copy_regions", self._h, *[r[k].ctypes.data_as(ctypes.c_void_p) for k in order])
        return r

    def num_slots(self) -> int:
        n = ctypes.c_int()
        nat.call("sbmp_kgmt_num_slots", self._h, ctypes.byref(n))
        return n.value

    def rng(self) -> np.ndarray:
        n = self.num_slots()
        out = np.zeros((n, 6), dtype=np.uint32)
        nat.call("sbmp_kgmt_copy_rng", self._h, out.ctypes.data_as(ctypes.c_void_p), n)
        return out

    def iter_log(self) -> np.ndarray:
        cnt = ctypes.c_int()
        nat.call("sbmp_kgmt_iter_log", self._h, None, 0, ctypes.byref(cnt))
        arr = (nat.IterRecord * max(1, cnt.value))()
        nat.call("sbmp_kgmt_iter_log", self._h, ctypes.cast(arr, ctypes.c_void_p), cnt.value, ctypes.byref(cnt))
        return np.array([[getattr(arr[i], k) for k in nat.ITER_FIELDS] for i in range(cnt.value)],
                        dtype=np.int64).reshape(-1, len(nat.ITER_FIELDS))

    def export_csv(self, directory: str) -> None:
        """The 13 CSV dumps of KGMT.cu:299-311."""
        nat.call("sbmp_kgmt_export_csv", self._h, directory.encode())

    def set_iteration_dump(self, directory: Optional[str]) -> None:
        """Per-iteration Data/<Kind>/<kind><itr>.csv dumps during plan() (KGMT.cu:263-290); None: off."""
        nat.call("sbmp_kgmt_set_iteration_dump", self._h, directory.encode() if directory else None)

    def kernel_stats(self) -> dict:
        cnt = ctypes.c_int()
        arr = (nat.KernelStat * 16)()
        nat.call("sbmp_kgmt_kernel_stats", self._h, ctypes.cast(arr, ctypes.c_void_p), 16, ctypes.byref(cnt))
        return {arr[i].name.decode(): (arr[i].launches, arr[i].totalMs) for i in range(min(cnt.value, 16))}

    def reset_kernel_stats(self) -> None:
        nat.call("sbmp_kgmt_reset_kernel_stats", self._h)

    OBSTACLE_FORMS = ("registers", "lds", "grid", "global")
    EXCHANGES = ("none", "oneshot", "collective")

    def path_info(self) -> dict:
        """The form of the hot path chosen at the last begin() (sbmp_kgmt_path_info)."""
        pi = nat.PathInfo()
        nat.call("sbmp_kgmt_path_info", self._h, ctypes.byref(pi))
        return {"form": "k_step" if pi.stepForm else "two-launch",
                "obstacle_form": self.OBSTACLE_FORMS[pi.obstacleForm] if 0 <= pi.obstacleForm < 4 else pi.obstacleForm,
                "resident_groups": pi.residentGroups, "needed_groups": pi.neededGroups,
                "exchange": self.EXCHANGES[pi.exchange] if 0 <= pi.exchange < 3 else pi.exchange,
                "nranks": pi.nranks, "rank": pi.rank, "rccl_nranks": pi.commRanks,
                "list_mirror": bool(pi.listMirror), "fused_exchange": bool(pi.fusedExchange),
                "oneshot_check": {0: "not run", 1: "passed", -1: "failed"}.get(pi.oneshotCheck, pi.oneshotCheck),
                "mirror_check": {0: "not run", 1: "passed", -1: "failed"}.get(pi.mirrorCheck, pi.mirrorCheck),
                "fused_check": {0: "not run", 1: "passed", -1: "failed"}.get(pi.fusedCheck, pi.fusedCheck),
                "row_table_lds": bool(pi.rowTableLds)}

    def kernel_samples(self, name: str) -> np.ndarray:
        """Per-launch durations (ms) of kernel `name` since the last reset_kernel_stats()."""
        cnt = ctypes.c_int()
        nat.call("sbmp_kgmt_kernel_samples", self._h, name.encode(), None, 0, ctypes.byref(cnt))
        out = np.zeros(max(1, cnt.value), dtype=np.float32)
        nat.call("sbmp_kgmt_kernel_samples", self._h, name.encode(), out.ctypes.data_as(ctypes.c_void_p),
                 cnt.value, ctypes.byref(cnt))
        return out[: cnt.value]

    def enqueue_delay(self, microseconds: float) -> None:
        """Hold the stream for a bounded time so the launches queued next run back to back."""
        nat.call("sbmp_kgmt_enqueue_delay", self._h, float(microseconds))

    def set_profiling(self, enabled: bool) -> None:
        nat.call("sbmp_kgmt_set_profiling", self._h, int(bool(enabled)))

    def state_hash(self) -> int:
        """64-bit digest of the replicated state (tree, tables, control blocks): equal on every rank."""
        h = ctypes.c_uint64()
        nat.call("sbmp_kgmt_state_hash", self._h, ctypes.byref(h))
        return int(h.value)

