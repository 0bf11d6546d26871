"""System / workspace configuration.

The reference hardcodes everything in demos/main.cu:19-46 and ships an empty
systems/car.yaml (yaml-cpp is linked but never called, CMakeLists.txt:10,47).
systems/*.yaml hold those constants and the benchmark workloads c1-c5; they are
read by the library's own parser (sbmp_load_system_config, csrc/config.cpp), the
same one the C++ demo and facade use, so Python needs no YAML package.
"""
from __future__ import annotations

import ctypes
import os

from . import _native as nat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYSTEMS = os.path.join(ROOT, "systems")

# reference demos/main.cu:33-45
DEMO_INITIAL = (5.0, 5.0, 0.0, 0.0, 0.0, 0.0, 0.0)
DEMO_GOAL = (2.0, 18.0, 0.0, 0.0, 0.0, 0.0, 0.0)

PLANNER_KEYS = ("width", "height", "N", "n", "numIterations", "maxTreeSize", "numDisc", "agentLength",
                "goalThreshold")


def load_system_config(path: str = os.path.join(SYSTEMS, "car.yaml")) -> dict:
    """Return {'planner': KGMT ctor kwargs, 'agent', 'samplesPerIteration', 'batchRule',
    'fixGNewClear', 'initial', 'goal', 'obstacles' (resolved path or None)}."""
    c = nat.SystemConfig()
    nat.call("sbmp_load_system_config", os.fspath(path).encode(), ctypes.byref(c))
    p = c.params
    obstacles = c.obstacles.decode()
    return {
        "planner": {k: getattr(p, k) for k in PLANNER_KEYS},
        "agent": "point" if p.agent == nat.SBMP_AGENT_POINT else "car",
        "samplesPerIteration": p.samplesPerIteration,
        "batchRule": "fill" if p.batchRule == nat.SBMP_BATCH_FILL else "reference",
        "fixGNewClear": bool(p.fixGNewClear),
        "initial": tuple(float(v) for v in c.initial),
        "goal": tuple(float(v) for v in c.goal),
        "obstacles": obstacles or None,
    }


def workload(name: str) -> dict:
    """The benchmark workload systems/<name>.yaml (c1-c5, BASELINE.json configs)."""
    return load_system_config(os.path.join(SYSTEMS, f"{name}.yaml"))
