"""LDS-add collisions of k_fold_r2 on the c3 workload's real children (diagnostics, GPU box).

Runs c3 for N iterations, reads the last iteration's children (sbmp_kgmt_copy_unexplored),
bins them like getR2 (the R2 cell; the valid bit does not change the word) and reports, for
the fold's lane layouts, how many lanes of one wave-level add share a word (the LDS
serialises them) and how many distinct words meet on one bank of a 32-lane group.
    python3 tools/fold_keys.py [N]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cells(st, W, N, n):
    R1 = W / N
    R2 = R1 / n
    x, y = st[:, 0], st[:, 1]
    cx, cy = np.floor(x / R1).astype(np.int64), np.floor(y / R1).astype(np.int64)
    ok = (cx >= 0) & (cx < N) & (cy >= 0) & (cy < N)
    r1 = cy * N + cx
    lx, ly = x - cx * R1, y - cy * R1
    sx, sy = np.floor(lx / R2).astype(np.int64), np.floor(ly / R2).astype(np.int64)
    ok &= (sx >= 0) & (sx < n) & (sy >= 0) & (sy < n)
    return np.where(ok, r1 * n * n + sy * n + sx, -1)


def layout_stats(key, lanes):
    """key[lanes]: one row per wave-level add (64 lanes)."""
    k = key[lanes]
    same, bankw = [], []
    for row in k:
        row = row[row >= 0]
        if len(row) == 0:
            continue
        _, c = np.unique(row, return_counts=True)
        same.append(c.max())
        worst = 0
        for g in (row[:32], row[32:]):
            if len(g) == 0:
                continue
            u = np.unique(g)
            worst = max(worst, np.bincount(u % 32, minlength=32).max())
        bankw.append(worst)
    return np.mean(same), np.percentile(same, 90), np.mean(bankw)


def main():
    its = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    from cudasbmp_amd import DeviceBuffer, read_obstacles_csv
    from cudasbmp_amd.config import workload
    from cudasbmp_amd.kgmt import KGMT
    cfg = workload("c3")
    obs = read_obstacles_csv(cfg["obstacles"])
    pl = dict(cfg["planner"])
    pl.update(numIterations=its + 2)
    k = KGMT(**pl, samplesPerIteration=262144, agent=cfg["agent"], batchRule=cfg["batchRule"], fixGNewClear=True)
    d_obs = DeviceBuffer(obs)
    k.begin(cfg["initial"], cfg["goal"], d_obs, len(obs), 20240807)
    k.enqueue(its)
    k.sync()
    st, par = k.unexplored()
    S = k.num_slots()
    st, par = st[:S], par[:S]
    W = pl.get("width", 20.0)
    key = cells(st, W, pl.get("N", 16), pl.get("n", 8))
    print(f"c3 after {its} iterations: {S} slots, {len(np.unique(key[key >= 0]))} distinct cells, "
          f"{len(np.unique(par))} parents")
    nS = S - S % 512
    # round-4 layout: lane L of the add j covers slot 8 L + j of a 512-slot window
    w = np.arange(nS).reshape(-1, 64, 8).transpose(0, 2, 1).reshape(-1, 64)
    print("consecutive 16-B pieces:  lanes on one word mean %.1f p90 %.0f, words on one bank %.1f" % layout_stats(key, w))
    # spread layout: lanes 1,024 slots apart
    per = 8192 * 8
    lanes = []
    for b in range(0, nS - per + 1, per):
        for wv in range(16):
            for j in range(64):
                u, e = divmod(j, 8)
                lanes.append(b + ((np.arange(64) * 16 + wv) * 8 + u) * 8 + e)
    print("lanes 1,024 slots apart:  lanes on one word mean %.1f p90 %.0f, words on one bank %.1f"
          % layout_stats(key, np.array(lanes)))
    # 8 regions (k_fold_r2): lane 8 g + e of wave wv, piece (u 16 + wv) 8 + e of region g
    lanes = []
    R = per // 8 // 8   # pieces per region of a 65,536-key group
    for b in range(0, nS - per + 1, per):
        for wv in range(16):
            for u in range(8):
                for j in range(8):
                    L = np.arange(64)
                    piece = (L >> 3) * R + (u * 16 + wv) * 8 + (L & 7)
                    lanes.append(b + piece * 8 + j)
    print("8 regions x 8 lanes:      lanes on one word mean %.1f p90 %.0f, words on one bank %.1f"
          % layout_stats(key, np.array(lanes)))
    rnd = np.random.default_rng(1).permutation(nS)[: (nS // 64) * 64].reshape(-1, 64)
    print("random slots:             lanes on one word mean %.1f p90 %.0f, words on one bank %.1f" % layout_stats(key, rnd))
    k.close()


if __name__ == "__main__":
    main()
