import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

OBSTACLES_CSV = os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv")
GOLDEN = os.path.join(ROOT, "tests", "golden")

# Demo configuration, reference demos/main.cu:19-46.
DEMO = dict(width=20.0, height=20.0, N=16, n=8, numIterations=100, maxTreeSize=30000, numDisc=10,
            agentLength=1.0, goalThreshold=0.5)
DEMO_INITIAL = (5.0, 5.0, 0.0, 0.0, 0.0, 0.0, 0.0)
DEMO_GOAL = (2.0, 18.0, 0.0, 0.0, 0.0, 0.0, 0.0)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def obstacles():
    # configurations/obstacles/obstacles.csv holds the reference's 5 boxes.
    return np.loadtxt(OBSTACLES_CSV, delimiter=",", dtype=np.float32).reshape(-1, 4)


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


def bits(a):
    """View float32 data as uint32 so comparisons are bit-exact and NaN-safe."""
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a
