"""ctypes binding of libsbmp.so (the C ABI in include/sbmp/sbmp.h).

The product path has no CPU fallback: if the HIP library is missing or fails to
load, every entry point raises NativeLibraryError.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libsbmp.so")

SBMP_OK = 0
SBMP_AGENT_CAR = 0
SBMP_AGENT_POINT = 1
SBMP_COMM_ID_BYTES = 128
SBMP_BATCH_REFERENCE = 0
SBMP_BATCH_FILL = 1


class NativeLibraryError(RuntimeError):
    pass


class SbmpError(RuntimeError):
    def __init__(self, status: int, func: str, msg: str):
        super().__init__(f"{func} failed with status {status}: {msg}")
        self.status = status


class KgmtParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_float), ("height", ctypes.c_float),
        ("N", ctypes.c_int), ("n", ctypes.c_int),
        ("numIterations", ctypes.c_int), ("maxTreeSize", ctypes.c_int), ("numDisc", ctypes.c_int),
        ("agentLength", ctypes.c_float), ("goalThreshold", ctypes.c_float),
        ("samplesPerIteration", ctypes.c_int), ("agent", ctypes.c_int), ("fixGNewClear", ctypes.c_int),
        ("device", ctypes.c_int), ("profileKernels", ctypes.c_int), ("batchRule", ctypes.c_int),
    ]


class PlanResult(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int), ("treeSize", ctypes.c_int), ("costToGoal", ctypes.c_float),
        ("goalIndex", ctypes.c_int), ("samplesGenerated", ctypes.c_longlong), ("accepted", ctypes.c_longlong),
        ("wallMs", ctypes.c_double), ("stalled", ctypes.c_int),
    ]


ITER_FIELDS = ("itr", "treeSizeBefore", "nG", "k", "nExp", "S", "A", "treeSizeAfter", "goalIdx")


class IterRecord(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ITER_FIELDS]


# sbmp_host_collectives (include/sbmp/sbmp.h): buffers are passed as raw addresses.
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


class HostCollectives(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allreduce_u64", ALLREDUCE_FN), ("allreduce_i32", ALLREDUCE_FN),
                ("allgather", ALLGATHER_FN)]


class SystemConfig(ctypes.Structure):   # sbmp_system_config
    _fields_ = [("params", KgmtParams), ("initial", ctypes.c_float * 7), ("goal", ctypes.c_float * 7),
                ("obstacles", ctypes.c_char * 1024)]


class ExpandBatchArgs(ctypes.Structure):   # sbmp_expand_batch_args
    _fields_ = [("count", ctypes.c_int), ("parents", ctypes.c_void_p), ("rng", ctypes.c_void_p),
                ("obstacles", ctypes.c_void_p), ("obstaclesCount", ctypes.c_int), ("agent", ctypes.c_int),
                ("numDisc", ctypes.c_int), ("agentLength", ctypes.c_float), ("width", ctypes.c_float),
                ("height", ctypes.c_float), ("N", ctypes.c_int), ("n", ctypes.c_int), ("R1Score", ctypes.c_void_p),
                ("R2Avail", ctypes.c_void_p), ("children", ctypes.c_void_p), ("valid", ctypes.c_void_p),
                ("r1", ctypes.c_void_p), ("r2", ctypes.c_void_p), ("accept", ctypes.c_void_p)]


class InsertBatchArgs(ctypes.Structure):   # sbmp_insert_batch_args
    _fields_ = [("slots", ctypes.c_int), ("gnew", ctypes.c_void_p), ("unexplored", ctypes.c_void_p),
                ("uParent", ctypes.c_void_p), ("samples", ctypes.c_void_p), ("parent", ctypes.c_void_p),
                ("costs", ctypes.c_void_p), ("treeSize", ctypes.c_int), ("maxTreeSize", ctypes.c_int),
                ("goalX", ctypes.c_float), ("goalY", ctypes.c_float), ("goalThreshold", ctypes.c_float),
                ("fixGNewClear", ctypes.c_int), ("inserted", ctypes.c_void_p), ("goalIndex", ctypes.c_void_p)]


class PathInfo(ctypes.Structure):   # sbmp_path_info
    _fields_ = [(n, ctypes.c_int) for n in ("stepForm", "obstacleForm", "residentGroups", "neededGroups", "exchange",
                                            "nranks", "rank", "commRanks", "listMirror",
                                            "fusedExchange", "oneshotCheck", "mirrorCheck", "fusedCheck", "rowTableLds")]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_longlong), ("totalMs", ctypes.c_double)]


# Every symbol include/sbmp/sbmp.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "sbmp_abi_version", "sbmp_status_string", "sbmp_last_error", "sbmp_kgmt_default_params",
    "sbmp_kgmt_create", "sbmp_kgmt_destroy", "sbmp_kgmt_plan", "sbmp_kgmt_begin", "sbmp_kgmt_step",
    "sbmp_kgmt_enqueue", "sbmp_kgmt_sync", "sbmp_kgmt_fold", "sbmp_kgmt_result", "sbmp_kgmt_stream", "sbmp_kgmt_copy_tree",
    "sbmp_kgmt_copy_unexplored", "sbmp_kgmt_copy_flags", "sbmp_kgmt_copy_regions", "sbmp_kgmt_num_slots",
    "sbmp_kgmt_copy_rng", "sbmp_kgmt_iter_log", "sbmp_kgmt_export_csv", "sbmp_kgmt_kernel_stats", "sbmp_kgmt_path_info",
    "sbmp_kgmt_reset_kernel_stats", "sbmp_kgmt_set_profiling", "sbmp_kgmt_state_hash", "sbmp_kgmt_kernel_samples", "sbmp_kgmt_enqueue_delay",
    "sbmp_read_obstacles_csv", "sbmp_device_upload_f32", "sbmp_device_free",
    "sbmp_device_count", "sbmp_comm_get_unique_id", "sbmp_kgmt_create_sharded", "sbmp_kgmt_create_local_group",
    "sbmp_kgmt_create_sharded_host", "sbmp_expand_batch", "sbmp_expand_batch_host", "sbmp_insert_batch",
    "sbmp_device_alloc", "sbmp_device_copy_to", "sbmp_device_copy_from", "sbmp_kgmt_set_iteration_dump",
    "sbmp_load_system_config",
    "sbmp_obstacle_grid_query", "sbmp_kgmt_solution_path", "sbmp_random_tree", "sbmp_hbm_copy_bandwidth",
)

_lib = None


def lib():
    """Load libsbmp.so (once).  Raises NativeLibraryError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -m cudasbmp_amd.build` (hipcc, gfx950). "
            "There is no CPU fallback for the planner.")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    vp, i, P = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER
    L.sbmp_abi_version.restype = i
    L.sbmp_status_string.restype = ctypes.c_char_p
    L.sbmp_status_string.argtypes = [i]
    L.sbmp_last_error.restype = ctypes.c_char_p
    sig = {
        "sbmp_kgmt_default_params": [P(KgmtParams)],
        "sbmp_load_system_config": [ctypes.c_char_p, P(SystemConfig)],
        "sbmp_kgmt_create": [P(KgmtParams), P(vp)],
        "sbmp_kgmt_create_sharded": [P(KgmtParams), vp, i, i, P(vp)],
        "sbmp_kgmt_create_local_group": [P(KgmtParams), i, P(vp)],
        "sbmp_kgmt_create_sharded_host": [P(KgmtParams), P(HostCollectives), i, i, P(vp)],
        "sbmp_expand_batch": [P(ExpandBatchArgs), vp],
        "sbmp_expand_batch_host": [P(ExpandBatchArgs)],
        "sbmp_insert_batch": [P(InsertBatchArgs), vp],
        "sbmp_device_alloc": [ctypes.c_size_t, P(vp)],
        "sbmp_device_copy_to": [vp, vp, ctypes.c_size_t],
        "sbmp_device_copy_from": [vp, vp, ctypes.c_size_t],
        "sbmp_comm_get_unique_id": [vp],
        "sbmp_kgmt_destroy": [vp],
        "sbmp_kgmt_plan": [vp, vp, vp, vp, i, ctypes.c_uint64, P(PlanResult)],
        "sbmp_kgmt_begin": [vp, vp, vp, vp, i, ctypes.c_uint64],
        "sbmp_kgmt_step": [vp, i, P(i)],
        "sbmp_kgmt_enqueue": [vp, i],
        "sbmp_kgmt_sync": [vp],
        "sbmp_kgmt_fold": [vp],
        "sbmp_kgmt_result": [vp, P(PlanResult)],
        "sbmp_kgmt_stream": [vp, P(vp)],
        "sbmp_kgmt_copy_tree": [vp, vp, vp, vp, i],
        "sbmp_kgmt_copy_unexplored": [vp, vp, vp, i],
        "sbmp_kgmt_copy_flags": [vp, vp, vp, i],
        "sbmp_kgmt_copy_regions": [vp] * 9,
        "sbmp_kgmt_num_slots": [vp, P(i)],
        "sbmp_kgmt_copy_rng": [vp, vp, i],
        "sbmp_kgmt_iter_log": [vp, vp, i, P(i)],
        "sbmp_kgmt_export_csv": [vp, ctypes.c_char_p],
        "sbmp_kgmt_set_iteration_dump": [vp, ctypes.c_char_p],
        "sbmp_kgmt_kernel_stats": [vp, vp, i, P(i)],
        "sbmp_kgmt_path_info": [vp, vp],
        "sbmp_kgmt_reset_kernel_stats": [vp],
        "sbmp_kgmt_set_profiling": [vp, i],
        "sbmp_kgmt_state_hash": [vp, P(ctypes.c_uint64)],
        "sbmp_kgmt_kernel_samples": [vp, ctypes.c_char_p, vp, i, P(i)],
        "sbmp_kgmt_enqueue_delay": [vp, ctypes.c_double],
        "sbmp_read_obstacles_csv": [ctypes.c_char_p, i, vp, i, P(i)],
        "sbmp_obstacle_grid_query": [vp, i, ctypes.c_float, ctypes.c_float, i, vp, i, vp, P(i)],
        "sbmp_kgmt_solution_path": [vp, i, vp, vp, vp, i, P(i)],
        "sbmp_random_tree": [i, i, vp, i, i, i, vp, ctypes.c_longlong, P(ctypes.c_float)],
        "sbmp_device_upload_f32": [vp, ctypes.c_size_t, P(vp)],
        "sbmp_device_free": [vp],
        "sbmp_device_count": [P(i)],
        "sbmp_hbm_copy_bandwidth": [ctypes.c_size_t, i, P(ctypes.c_double)],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = i
    _lib = L
    return _lib


def check(status: int, func: str) -> None:
    if status != SBMP_OK:
        msg = lib().sbmp_last_error().decode(errors="replace")
        raise SbmpError(status, func, msg)


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
