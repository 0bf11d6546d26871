"""Interleaved A/B of planner variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/ab_expand.py [--rounds 6] [--iters 40]

Each variant is a planner created with a different SBMP_EXPAND_VARIANT; every
round times `iters` steady-state iterations of the c3 workload per variant.
Prints per-variant median/min step time and the median k_expand duration.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv  # noqa: E402


def make(env, iters_total):
    for kv in env.split(","):
        if kv:
            key, val = kv.split("=")
            os.environ[key] = val
    k = KGMT(20.0, 20.0, 16, 8, iters_total, 1 << 24, 10, 1.0, 0.0, samplesPerIteration=262144,
             batchRule="fill", fixGNewClear=True)   # bench workload (bench.py --gnew-clear complete)
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--configs", default="SBMP_EXPAND_VARIANT=1;SBMP_EXPAND_VARIANT=3",
                    help="';'-separated configurations, each a ','-separated list of ENV=value")
    a = ap.parse_args()
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    d_obs = DeviceBuffer(obs)
    variants = a.configs.split(";")
    res = {v: [] for v in variants}
    kexp = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            k = make(v, 20 + 2 * a.iters + 2)
            k.begin((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), d_obs, len(obs), 20240807)
            k.enqueue(20)
            k.sync()
            prof_timed = os.environ.get("SBMP_PROFILE_TIMED") == "1"
            k.set_profiling(prof_timed)
            k.reset_kernel_stats()
            t0 = time.perf_counter()
            k.enqueue(a.iters)
            k.sync()
            res[v].append((time.perf_counter() - t0) / a.iters * 1e6)
            if not prof_timed:
                k.set_profiling(True)
                k.enqueue_delay(4000.0)
                k.enqueue(a.iters)
                k.sync()
            st = k.kernel_stats()
            n, ms = st["k_expand"]
            kexp[v].append(ms / max(1, n) * 1e3)
            os.environ.pop("SBMP_PROFILE_TIMED", None)
            k.close()
    for v in variants:
        print(f"variant {v}: step median {np.median(res[v]):.2f} us min {np.min(res[v]):.2f} us; "
              f"k_expand median {np.median(kexp[v]):.2f} us")


if __name__ == "__main__":
    main()
