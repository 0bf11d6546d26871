"""Per-wave Euler-loop extras of one c3 iteration, from the oracle (host analysis).

    python tools/cull_stats.py [iteration] [block ...]

For every 64-slot wave of k_step(t): the boxes its cull keeps (kgmt_device.h
wave_cull: the union of the lanes' squares of half-width T|v0| + |a|T^2/2 around
the parent), whether it keeps the workspace-bounds test, and whether the Payne-Hanek
check stays on (car_theta_bounded) -- the per-step work beyond the ~40 VALU of a
culled step.  Replays the bench's c3 workload (complete clear, fill rule, seed
20240807) in the oracle up to iteration t.
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oracle.pyoracle import Oracle, PlannerConfig  # noqa: E402

t = int(sys.argv[1]) if len(sys.argv) > 1 else 20
blocks = [int(b) for b in sys.argv[2:]]
cfg = PlannerConfig(maxTreeSize=1 << 24, samplesPerIteration=262144, goalThreshold=0.0, fixGNewClear=1,
                    batchRule=1, numIterations=100)
obs = np.loadtxt("configurations/obstacles/obstacles.csv", delimiter=",", dtype=np.float32).reshape(-1, 4)
o = Oracle(cfg, threads=8)
o.begin([5, 5, 0, 0, 0, 0, 0], [2, 18, 0, 0, 0, 0, 0], obs, 20240807)
for _ in range(t):
    o.step()
tree, _, _ = o.tree()
us, upar = o.unexplored()
logs = o.iter_logs()
S = int(logs[-1][list(range(len(logs[-1])))].tolist()[0] * 0 + (upar >= 0).sum())
n = (upar[:262144] >= 0).sum()
par = upar[:n]
p = tree[par]            # x, y, theta, v (, ...)
a, T = us[:n, 4], us[:n, 6]
r = T * np.abs(p[:, 3]) + 0.5 * np.abs(a) * T * T
r = r * 1.0001 + 1e-3
W = 20.0
nw = n // 64
kept = np.zeros(nw, dtype=int)
bounds = np.zeros(nw, dtype=bool)
for w in range(nw):
    sl = slice(64 * w, 64 * w + 64)
    x0, y0, rr = p[sl, 0], p[sl, 1], r[sl]
    mnx, mny, mxx, mxy = x0 - rr, y0 - rr, x0 + rr, y0 + rr
    bounds[w] = not np.all((mnx > 0) & (mny > 0) & (mxx < W) & (mxy < W))
    for ob in obs:
        sep = np.maximum.reduce([ob[0] - mxx, ob[1] - mxy, mnx - ob[2], mny - ob[3]])
        kept[w] += bool(np.any(sep < 0))
extra = kept * 5 + bounds * 5
print(f"iteration {t}: {n} children, {nw} waves")
print("boxes kept per wave:", np.bincount(kept, minlength=6).tolist())
print("waves with the bounds test:", int(bounds.sum()))
print("extra VALU per step: p50 %d p90 %d p99 %d max %d" % tuple(np.percentile(extra, [50, 90, 99, 100])))
print("mean |v0| %.2f, mean square half-width %.2f" % (np.abs(p[:, 3]).mean(), r.mean()))
for b in blocks:
    print("block", b, "waves kept", kept[4 * (b - 1):4 * b].tolist(), "bounds", bounds[4 * (b - 1):4 * b].tolist())


def cull(frac):
    """kept boxes and bounds flag per wave for squares of the displacement bound at frac * T"""
    tt = T * frac
    rr_all = (tt * np.abs(p[:, 3]) + 0.5 * np.abs(a) * tt * tt) * 1.0001 + 1e-3
    k = np.zeros(nw, dtype=int)
    bd = np.zeros(nw, dtype=bool)
    for w in range(nw):
        sl = slice(64 * w, 64 * w + 64)
        x0, y0, rr = p[sl, 0], p[sl, 1], rr_all[sl]
        mnx, mny, mxx, mxy = x0 - rr, y0 - rr, x0 + rr, y0 + rr
        bd[w] = not np.all((mnx > 0) & (mny > 0) & (mxx < W) & (mxy < W))
        for ob in obs:
            sep = np.maximum.reduce([ob[0] - mxx, ob[1] - mxy, mnx - ob[2], mny - ob[3]])
            k[w] += bool(np.any(sep < 0))
    return k, bd


def step_cost(k, bd):
    return 38 + np.where(k > 0, 6 + 5 * k, 0) + 5 * bd


full = step_cost(kept, bounds)
print("VALU per wave in the loop, one cull: mean %.0f" % (10 * full).mean())
for parts in (2, 3, 5):
    tot = np.zeros(nw)
    for q in range(parts):
        k, bd = cull((q + 1) / parts)
        tot += step_cost(k, bd) * (10 / parts)
    extra = (parts - 1) * 36
    print(f"{parts} culls (+{extra} VALU): mean {tot.mean() + extra:.0f}")

# deaths per wave: invalid children (collision or out of bounds) end their loop early;
# the state replay of the oracle gives each child's validity, not its step, so count
# the waves holding any invalid child
_, gnew = o.flags()
print("children flagged valid: %.1f%%" % (100.0 * gnew[:n].mean()))
