"""Diagnostic: stepwise demo plan against the oracle, printing the first differing
rows / columns of each array (used to bisect kernel-form differences, e.g.
SBMP_STEP=0 python tools/diag_loop.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, bits  # noqa: E402
from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv  # noqa: E402
from oracle.pyoracle import Oracle, PlannerConfig  # noqa: E402


def show(name, a, b, n=4):
    a, b = bits(np.asarray(a)), bits(np.asarray(b))
    a2, b2 = a.reshape(len(a), -1), b.reshape(len(b), -1)
    rows = np.nonzero((a2 != b2).any(axis=1))[0]
    if len(rows) == 0:
        print(f"  {name}: equal")
        return
    print(f"  {name}: {len(rows)} rows differ, first {rows[:8].tolist()}")
    for r in rows[:n]:
        cols = np.nonzero(a2[r] != b2[r])[0].tolist()
        print(f"    row {r} cols {cols} gpu {a2[r].view(np.float32).tolist()} oracle {b2[r].view(np.float32).tolist()}")


def main():
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    d_obs = DeviceBuffer(obs)
    g = KGMT(**DEMO)
    o = Oracle(PlannerConfig(**DEMO), threads=8)
    g.begin(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obs), 42)
    o.begin(DEMO_INITIAL, DEMO_GOAL, obs, 42)
    for it in range(1, 4):
        g.step(1)
        o.step()
        print(f"iteration {it}")
        lg, lo = g.iter_log(), o.iter_logs()
        print("  log equal" if np.array_equal(lg, lo) else f"  logs\n{lg}\n{lo}")
        sg, pg, cg = g.tree()
        so, po, co = o.tree()
        show("parents", pg, po)
        show("samples", sg, so)
        show("costs", cg, co)
        ug, upg = g.unexplored()
        uo, upo = o.unexplored()
        show("uParent", upg, upo)
        show("unexplored", ug, uo)
        show("rng", g.rng(), o.rng())
        Gg, GNg = g.flags()
        Go, GNo = o.flags()
        show("GNew", GNg, GNo)
        rg, ro = g.regions(), o.regions()
        for k in ro:
            show(k, rg[k], ro[k], n=2)


if __name__ == "__main__":
    main()
