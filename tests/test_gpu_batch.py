"""The step-level entry points on the GPU, each against the CPU oracle:
  sbmp_expand_batch  the public headers' propagateAndCheck / getR1 / getR2 + accept test in
                     a device kernel vs oracle_expand_batch (bit-exact children, flags,
                     cells, RNG states);
  sbmp_insert_batch  exclusive_scan(GNew) + findInd + updateG vs the oracle's numpy updateG
                     (KGMT.cu:221-249, 540-593): rows, parents, costs, the D6 clear, A, goal.
"""
import numpy as np
import pytest

from conftest import bits
from test_batch import _batch, _obstacle_sets

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("agent", ["car", "point"])
@pytest.mark.parametrize("obs_name", ["demo", "none", "c5"])
@pytest.mark.parametrize("numDisc,L", [(10, 1.0), (7, 1.3)])
def test_expand_batch_device_matches_oracle(agent, obs_name, numDisc, L, obstacles, oracle_lib):
    from cudasbmp_amd.batch import expand_batch
    from oracle.pyoracle import PlannerConfig, expand_batch as oracle_expand
    obs = _obstacle_sets(obstacles)[obs_name]
    k = 65536 if obs_name != "c5" else 4096
    parents, states = _batch(k, 11 + numDisc, agent)
    rng = np.random.default_rng(3)
    score = rng.uniform(0, 0.02, size=256).astype(np.float32)
    avail = (rng.uniform(size=256 * 64) < 0.5).astype(np.int32)
    g = expand_batch(parents, states, obs, numDisc=numDisc, agentLength=L, agent=agent, R1Score=score,
                     R2Avail=avail)
    o = oracle_expand(PlannerConfig(numDisc=numDisc, agentLength=L, agent=1 if agent == "point" else 0), obs,
                      parents, states, score, avail, threads=16)
    assert np.array_equal(bits(g["children"]), bits(o["children"]))
    for key in ("valid", "r1", "r2", "accept", "rng"):
        assert np.array_equal(g[key], o[key]), key


@pytest.mark.parametrize("slots,M,treeSize,frac,fix", [
    (262144, 1 << 20, 5000, 0.004, True),     # c3-like steady state: ~1,000 accepted of 262,144
    (262144, 1 << 20, 1, 0.9, False),        # iteration-1-like: most slots accepted, partial clear (D6)
    (4096, 3000, 2900, 0.5, False),          # tree fills: rows past M dropped (D13), grid limit
    (1000, 30000, 100, 0.0, False),          # nothing accepted
    (33, 64, 10, 1.0, False),                # ragged slot count, M/32 = 2 blocks of updateG
])
def test_insert_batch_device_matches_oracle(slots, M, treeSize, frac, fix):
    from cudasbmp_amd.batch import insert_batch
    from oracle.pyoracle import insert_batch as oracle_insert
    rng = np.random.default_rng(slots + M)
    gnew = (rng.uniform(size=slots) < frac).astype(np.uint8)
    unexplored = rng.uniform(0, 20, size=(slots, 7)).astype(np.float32)
    uParent = rng.integers(0, treeSize, size=slots).astype(np.int32)
    samples = np.zeros((M, 7), np.float32)
    parent = np.full(M, -1, np.int32)
    costs = np.zeros(M, np.float32)
    costs[:treeSize] = rng.uniform(0, 30, size=treeSize).astype(np.float32)
    goal, r = (7.0, 11.0), 0.8
    g = insert_batch(gnew, unexplored, uParent, samples, parent, costs, treeSize, goal, r, fix)
    o = oracle_insert(gnew, unexplored, uParent, samples, parent, costs, treeSize, goal, r, fix)
    assert np.array_equal(bits(g[0]), bits(o[0])) and np.array_equal(g[1], o[1])
    assert np.array_equal(bits(g[2]), bits(o[2])) and np.array_equal(g[3], o[3])
    assert g[4] == o[4] and g[5] == o[5]
