"""Host-side costs around the bench's timed window (GPU box): enqueue(K), fold(),
sync() and the whole window, medians over reps, for the c3 workload.
    python tools/host_overhead.py [K] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import DeviceBuffer, read_obstacles_csv  # noqa: E402
from cudasbmp_amd.config import workload  # noqa: E402
from cudasbmp_amd.kgmt import KGMT  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = workload("c3")
    pl = dict(cfg["planner"])
    pl.update(numIterations=5 + K * reps + 2)
    k = KGMT(**pl, samplesPerIteration=cfg["samplesPerIteration"], agent=cfg["agent"], batchRule=cfg["batchRule"],
             fixGNewClear=True)
    obs = read_obstacles_csv(cfg["obstacles"])
    d_obs = DeviceBuffer(obs)
    k.begin(cfg["initial"], cfg["goal"], d_obs, len(obs), 20240807)
    k.enqueue(5)
    k.fold()
    k.sync()
    rows = []
    for _ in range(reps):
        k.sync()
        t0 = time.perf_counter()
        k.enqueue(K)
        t1 = time.perf_counter()
        k.fold()
        t2 = time.perf_counter()
        k.sync()
        t3 = time.perf_counter()
        rows.append([t1 - t0, t2 - t1, t3 - t2, t3 - t0])
    m = np.median(np.array(rows), axis=0) * 1e6
    print(f"K={K} SBMP_SPIN={os.environ.get('SBMP_SPIN', '1')}: enqueue {m[0]:.1f} us, fold {m[1]:.1f} us, "
          f"sync {m[2]:.1f} us, window {m[3]:.1f} us ({m[3] / K:.2f} us per step)")


if __name__ == "__main__":
    main()
