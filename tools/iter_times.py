"""Per-iteration k_step durations of the c3 bench workload next to the iteration log
(frontier, children per parent, accepted), over iterations 1..N (GPU box):
    python tools/iter_times.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import DeviceBuffer, read_obstacles_csv  # noqa: E402
from cudasbmp_amd.config import workload  # noqa: E402
from cudasbmp_amd.kgmt import KGMT  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    cfg = workload("c3")
    obs = read_obstacles_csv(cfg["obstacles"])
    pl = dict(cfg["planner"])
    pl.update(numIterations=n + 2)
    k = KGMT(**pl, samplesPerIteration=cfg["samplesPerIteration"], agent=cfg["agent"], batchRule=cfg["batchRule"],
             fixGNewClear=True)
    d_obs = DeviceBuffer(obs)
    k.begin(cfg["initial"], cfg["goal"], d_obs, len(obs), 20240807)
    k.set_profiling(True)
    k.reset_kernel_stats()
    k.enqueue_delay(4000.0)
    k.enqueue(n)
    k.sync()
    us = [1e3 * v for v in k.kernel_samples("k_step")]
    log = k.iter_log()
    print(" t   treeSize     nG     k        S       A    k_step us")
    for i, row in enumerate(log[:n]):
        print(f"{int(row[0]):3d} {int(row[1]):9d} {int(row[2]):6d} {int(row[3]):5d} {int(row[5]):8d} {int(row[6]):7d}  "
              f"{us[i] if i < len(us) else float('nan'):8.2f}")


if __name__ == "__main__":
    main()
