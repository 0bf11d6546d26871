"""TTFS probe (GPU box): plan() on the reference demo, seeds 1..10, against enqueueing exactly the
iterations each seed needs and one synchronisation.  python3 tools/ttfs_probe.py"""
import time, numpy as np, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv
obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
d_obs = DeviceBuffer(obs)
INIT = (5, 5, 0, 0, 0, 0, 0); GOAL = (2, 18, 0, 0, 0, 0, 0)
k = KGMT(20.0, 20.0, 16, 8, 100, 30000, 10, 1.0, 0.5, agent="car")
k.plan(INIT, GOAL, d_obs, len(obs), seed=1000)
res = {"plan": [], "enq_exact": [], "iters": []}
for seed in range(1, 11):
    r = k.plan(INIT, GOAL, d_obs, len(obs), seed=seed)
    res["plan"].append(r.wallMs); res["iters"].append(r.iterations)
for seed in range(1, 11):
    n = res["iters"][seed - 1]
    k.begin(INIT, GOAL, d_obs, len(obs), seed)
    t0 = time.perf_counter()
    k.enqueue(n + 1)
    k.sync()
    res["enq_exact"].append((time.perf_counter() - t0) * 1e3)
for kk, v in res.items():
    print(kk, np.round(v, 4).tolist(), "median", np.median(v))
