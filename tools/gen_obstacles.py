"""Synthetic obstacle field of config c5 (BASELINE.json configs[4]).

    python tools/gen_obstacles.py > configurations/obstacles/obstacles_c5.csv

10,000 axis-aligned boxes in the 20 x 20 demo workspace from splitmix64 (seed
20240807): centre U[0, 20)^2, half-extents U[0.02, 0.08) per axis, a box is
rejected when it comes within 1.0 of the demo start (5, 5) or goal (2, 18)
(reference demos/main.cu:39-45), so both stay reachable.  Rows are
xmin,ymin,xmax,ymax, the reference's obstacles.csv layout (helper.cu:11-34), each
value the float32 the planner will hold, printed to round-trip exactly.
"""
import argparse

import numpy as np

MASK = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & MASK

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        return lo + (hi - lo) * ((self.next() >> 11) * (1.0 / (1 << 53)))


def box_point_distance(b, px, py):
    dx = max(b[0] - px, 0.0, px - b[2])
    dy = max(b[1] - py, 0.0, py - b[3])
    return (dx * dx + dy * dy) ** 0.5


def generate(n=10000, seed=20240807, width=20.0, height=20.0, keep_clear=((5.0, 5.0), (2.0, 18.0)), clearance=1.0):
    rng = SplitMix64(seed)
    out = []
    while len(out) < n:
        cx, cy = rng.uniform(0.0, width), rng.uniform(0.0, height)
        hx, hy = rng.uniform(0.02, 0.08), rng.uniform(0.02, 0.08)
        b = [float(np.float32(v)) for v in (cx - hx, cy - hy, cx + hx, cy + hy)]
        if any(box_point_distance(b, px, py) < clearance for px, py in keep_clear):
            continue
        out.append(b)
    return np.array(out, dtype=np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=20240807)
    a = ap.parse_args()
    for b in generate(a.n, a.seed):
        print(",".join(np.format_float_positional(np.float32(v), unique=True, trim="-") for v in b))


if __name__ == "__main__":
    main()
