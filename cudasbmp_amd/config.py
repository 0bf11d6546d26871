"""System / workspace configuration.

The reference hardcodes everything in demos/main.cu:19-46 and ships an empty
systems/car.yaml (yaml-cpp is linked but never called, CMakeLists.txt:10,47).
This module reads systems/*.yaml (populated from main.cu's constants) so a
configuration can be selected without recompiling.
"""
from __future__ import annotations

import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# reference demos/main.cu:33-45
DEMO_INITIAL = (5.0, 5.0, 0.0, 0.0, 0.0, 0.0, 0.0)
DEMO_GOAL = (2.0, 18.0, 0.0, 0.0, 0.0, 0.0, 0.0)

PLANNER_KEYS = ("width", "height", "N", "n", "numIterations", "maxTreeSize", "numDisc", "agentLength",
                "goalThreshold")


def load_system_config(path: str = os.path.join(ROOT, "systems", "car.yaml")) -> dict:
    """Return {'planner': ctor kwargs, 'agent', 'initial', 'goal', 'obstacles' (path)}."""
    with open(path) as f:
        raw = yaml.safe_load(f) or {}
    missing = [k for k in PLANNER_KEYS if k not in raw]
    if missing:
        raise ValueError(f"{path}: missing keys {missing}")
    base = os.path.dirname(os.path.abspath(path))
    obstacles = raw.get("obstacles")
    if obstacles and not os.path.isabs(obstacles):
        obstacles = os.path.normpath(os.path.join(base, obstacles))
    return {
        "planner": {k: raw[k] for k in PLANNER_KEYS},
        "agent": raw.get("agent", "car"),
        "initial": tuple(float(v) for v in raw.get("initial", DEMO_INITIAL)),
        "goal": tuple(float(v) for v in raw.get("goal", DEMO_GOAL)),
        "obstacles": obstacles,
    }
