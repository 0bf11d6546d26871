import time, sys, os
ROOT = "/root/repo" if os.path.exists("/root/repo/cudasbmp_amd") else os.getcwd()
sys.path.insert(0, ROOT)
from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv
obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
d_obs = DeviceBuffer(obs)
k = KGMT(20.0, 20.0, 16, 8, 400, 30000, 10, 1.0, 0.0, agent="car")   # goal disabled: every iteration runs
for rep in range(3):
    k.begin((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), d_obs, len(obs), 7)
    t0 = time.perf_counter(); k.enqueue(100); t1 = time.perf_counter(); k.sync(); t2 = time.perf_counter()
    print(f"enqueue(100): host {1e6*(t1-t0)/100:.2f} us per launch, to sync {1e6*(t2-t0)/100:.2f} us per iteration")
