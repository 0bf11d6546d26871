"""The public device-function headers (include/sbmp/propagator.h, collision.h, grid.h,
xorwow.h) compiled for the host, through sbmp_expand_batch_host, against the CPU
oracle's independent restatement (oracle_expand_batch): children, validity, region
cells, accept flags and RNG states bit-exact.  No GPU needed; tests/test_gpu_batch.py
runs the same batches through the device kernel.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, bits


def _batch(k, seed, agent="car"):
    rng = np.random.default_rng(seed)
    parents = np.zeros((k, 7), dtype=np.float32)
    parents[:, 0:2] = rng.uniform(0.5, 19.5, size=(k, 2))
    parents[:, 2] = rng.uniform(-40, 40, size=k)        # theta: several turns, both signs
    parents[:, 3] = rng.uniform(-8, 8, size=k) if agent == "car" else 0.0
    parents[: k // 16, 2] = rng.uniform(-3e5, 3e5, size=k // 16)   # Payne-Hanek range
    states = rng.integers(0, 2**32, size=(k, 6), dtype=np.uint64).astype(np.uint32)
    return parents, states


def _obstacle_sets(obstacles):
    c5 = np.loadtxt(os.path.join(ROOT, "configurations", "obstacles", "obstacles_c5.csv"), delimiter=",",
                    dtype=np.float32).reshape(-1, 4)
    return {"demo": obstacles, "none": np.zeros((0, 4), np.float32), "c5": c5}


@pytest.mark.parametrize("agent", ["car", "point"])
@pytest.mark.parametrize("obs_name", ["demo", "none", "c5"])
@pytest.mark.parametrize("numDisc,L", [(10, 1.0), (7, 1.3)])
def test_expand_batch_host_matches_oracle(agent, obs_name, numDisc, L, obstacles, oracle_lib):
    from cudasbmp_amd.batch import expand_batch
    from oracle.pyoracle import PlannerConfig, expand_batch as oracle_expand
    obs = _obstacle_sets(obstacles)[obs_name]
    k = 2048 if obs_name != "c5" else 512
    parents, states = _batch(k, 11 + numDisc, agent)
    rng = np.random.default_rng(3)
    score = rng.uniform(0, 0.02, size=256).astype(np.float32)
    avail = (rng.uniform(size=256 * 64) < 0.5).astype(np.int32)
    g = expand_batch(parents, states, obs, numDisc=numDisc, agentLength=L, agent=agent, R1Score=score,
                     R2Avail=avail, device=False)
    cfg = PlannerConfig(numDisc=numDisc, agentLength=L, agent=1 if agent == "point" else 0)
    o = oracle_expand(cfg, obs, parents, states, score, avail)
    assert np.array_equal(bits(g["children"]), bits(o["children"]))
    for key in ("valid", "r1", "r2", "accept", "rng"):
        assert np.array_equal(g[key], o[key]), key
    assert 0 < g["valid"].sum() < k and g["accept"].sum() > 0


def test_expand_batch_host_without_scores(obstacles, oracle_lib):
    """No R1Score: no accept draw (the RNG advances by the three control draws only)."""
    from cudasbmp_amd.batch import expand_batch
    from oracle.pyoracle import PlannerConfig, expand_batch as oracle_expand
    parents, states = _batch(256, 5)
    g = expand_batch(parents, states, obstacles, device=False)
    o = oracle_expand(PlannerConfig(), obstacles, parents, states)
    assert np.array_equal(g["rng"], o["rng"]) and not g["accept"].any()
    assert np.array_equal(bits(g["children"]), bits(o["children"]))


def test_insert_batch_restatement_properties():
    """The oracle's numpy updateG (the checker of sbmp_insert_batch): slot order, the
    updateG grid limit, D13 and the D6 clear, on a small hand-checked case."""
    from oracle.pyoracle import insert_batch
    M = 64
    samples = np.zeros((M, 7), np.float32)
    parent = np.full(M, -1, np.int32)
    costs = np.zeros(M, np.float32)
    costs[0] = 1.5
    slots = 80
    gnew = np.zeros(slots, np.uint8)
    gnew[[3, 5, 40, 70]] = 1
    unexplored = np.arange(slots * 7, dtype=np.float32).reshape(slots, 7) / 100.0
    uParent = np.zeros(slots, np.int32)
    s, p, c, gn, A, goal = insert_batch(gnew, unexplored, uParent, samples, parent, costs, 62, (0.36, 0.37), 0.1)
    assert A == 4
    assert p[62] == 0 and p[63] == 0                       # slots 3, 5 -> rows 62, 63; rows >= M dropped
    assert np.array_equal(s[62], unexplored[3]) and np.array_equal(s[63], unexplored[5])
    assert c[62] == np.float32(1.5) + unexplored[3, 6]
    assert gn[:64].sum() == 0 and gn[70] == 1              # grid = min(4, 64/32) = 2: GNew[0..64) cleared
    assert goal == 63                                      # slot 5's child (0.35, 0.36) is within 0.1 of the goal; slot 3's is not
