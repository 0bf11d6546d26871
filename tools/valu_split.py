"""VALU / SALU per k_step wave against the Euler step count (diagnostics, GPU box).

Runs the c3 workload with numDisc = N (argument) for 30 iterations; under
    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -d <out> -o run --output-format csv -- python3 tools/valu_split.py N
the per-wave counts at N = 1, 5, 10 split k_step's instructions into the Euler loop's
(the slope) and everything else (the intercept).
    python3 tools/valu_split.py sum <out_N1> <out_N5> <out_N10>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(nd):
    from cudasbmp_amd import DeviceBuffer, read_obstacles_csv
    from cudasbmp_amd.config import workload
    from cudasbmp_amd.kgmt import KGMT
    cfg = workload("c3")
    obs = read_obstacles_csv(cfg["obstacles"])
    pl = dict(cfg["planner"])
    pl.update(numIterations=32, numDisc=nd)
    k = KGMT(**pl, samplesPerIteration=262144, agent=cfg["agent"], batchRule=cfg["batchRule"], fixGNewClear=True)
    d_obs = DeviceBuffer(obs)
    k.begin(cfg["initial"], cfg["goal"], d_obs, len(obs), 20240807)
    k.enqueue(30)
    k.sync()
    k.close()


def summarize(dirs):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_workload import per_dispatch
    for dpath in dirs:
        c, _ = per_dispatch(dpath)
        w = np.array(c["SQ_WAVES"][10:30])
        v = np.array(c["SQ_INSTS_VALU"][10:30]) / w
        s = np.array(c["SQ_INSTS_SALU"][10:30]) / w
        print(f"{dpath}: VALU per wave {v.mean():.1f}, SALU per wave {s.mean():.1f} (iterations 11-30)")


if __name__ == "__main__":
    if sys.argv[1] == "sum":
        summarize(sys.argv[2:])
    else:
        run(int(sys.argv[1]))
