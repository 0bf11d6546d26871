"""cudasbmp_amd — MI355X-native KGMT kinodynamic planner (drop-in for nipe1783/cudaSBMP's KGMT).

The hot path (expand -> propagate -> collision-check -> bin -> accept -> insert)
is hand-written HIP for gfx950 in csrc/, exposed through the C ABI in
include/sbmp/sbmp.h (libsbmp.so).  This package is the Python host mirror of
the reference's KGMT interface; it has no CPU fallback.
"""
from ._native import NativeLibraryError, SbmpError, LIB_PATH  # noqa: F401
from .kgmt import KGMT, DeviceBuffer, read_obstacles_csv, device_count, reference_seed_from_time, random_tree  # noqa: F401,E501
from .config import load_system_config, DEMO_INITIAL, DEMO_GOAL  # noqa: F401

__all__ = ["KGMT", "DeviceBuffer", "read_obstacles_csv", "device_count", "reference_seed_from_time", "random_tree",
           "load_system_config", "DEMO_INITIAL", "DEMO_GOAL", "NativeLibraryError", "SbmpError", "LIB_PATH"]
