"""Regenerate tests/golden/oracle_fixtures.json from the CPU oracle.

    python tests/golden/make_oracle_fixtures.py

The reference ships no test vectors, so these fixtures pin the
oracle against regressions: for each case the iteration log, the outcome, a few
tree rows as exact float32 bit patterns, RNG states of selected slots, and
SHA-256 digests of every state array in the reference's layout.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.pyoracle import Oracle, PlannerConfig, build  # noqa: E402

INIT = (5.0, 5.0, 0.0, 0.0, 0.0, 0.0, 0.0)
GOAL = (2.0, 18.0, 0.0, 0.0, 0.0, 0.0, 0.0)

CASES = {
    "demo_seed1": (dict(), 1),
    "demo_seed2": (dict(), 2),
    "demo_seed3": (dict(), 3),
    "demo_seed1723000000": (dict(), 1723000000),
    "capped_4096": (dict(samplesPerIteration=4096, maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 99),
    "fill_8192": (dict(samplesPerIteration=8192, batchRule=1, maxTreeSize=300000, numIterations=12,
                       goalThreshold=0.0), 99),
    "point_demo": (dict(agent=1), 5),
    "tiny_tree_700": (dict(maxTreeSize=700, numIterations=50), 99),
}


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_case(kw, seed, obstacles):
    o = Oracle(PlannerConfig(**kw), threads=8)
    o.plan(INIT, GOAL, obstacles, seed)
    info = o.info()
    s, p, c = o.tree()
    us, up = o.unexplored()
    g, gn = o.flags()
    reg = o.regions()
    rng = o.rng()
    n = min(info["treeSize"], len(p))
    rows = [0, 1, 2, n // 2, n - 1]
    slots = [i for i in (0, 1, 31, 32, 255, 256, len(rng) - 1) if i < len(rng)]
    return {
        "config": kw, "seed": seed,
        "iterations": info["iterations"], "treeSize": info["treeSize"], "goalIdx": info["goalIdx"],
        "costToGoal_bits": int(np.float32(info["costToGoal"]).view(np.uint32)),
        "samples": info["samples"],
        "iter_log": o.iter_logs().tolist(),
        "rows": {str(r): {"sample_bits": s[r].view(np.uint32).tolist(), "parent": int(p[r]),
                          "cost_bits": int(c[r:r + 1].view(np.uint32)[0])} for r in rows},
        "rng": {str(i): rng[i].tolist() for i in slots},
        "sha256": {"samples": digest(s), "parents": digest(p), "costs": digest(c), "unexplored": digest(us),
                   "uParent": digest(up), "G": digest(g), "GNew": digest(gn), "rng": digest(rng),
                   **{k: digest(v) for k, v in reg.items()}},
    }


def main():
    build()
    obstacles = np.loadtxt(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"),
                           delimiter=",", dtype=np.float32).reshape(-1, 4)
    out = {"generator": "tests/golden/make_oracle_fixtures.py", "initial": INIT, "goal": GOAL, "cases": {}}
    for name, (kw, seed) in CASES.items():
        out["cases"][name] = run_case(kw, seed, obstacles)
        print(name, out["cases"][name]["iterations"], out["cases"][name]["treeSize"])
    with open(os.path.join(HERE, "oracle_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
