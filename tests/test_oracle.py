"""CPU oracle (oracle/kgmt_oracle.cpp) pinned three ways, no GPU needed:

1. Golden fixtures (tests/golden/oracle_fixtures.json, made by
   tests/golden/make_oracle_fixtures.py): iteration logs, outcomes, float32 bit
   patterns and digests of every state array for 8 configurations.  The reference
   ships no vectors, so these catch regressions of the restatement.
2. The reference's RNG-independent invariants on demo runs
   (demos/main.cu:19-46): every tree row replays from its parent and controls
   (statePropagator.cu:5-76), parents precede children, costs accumulate
   (KGMT.cu:572,586), controls lie in the sampled ranges (statePropagator.cu:17-19)
   and the region counters balance (KGMT.cu:392-411).
3. The sharded protocol (slot-owning ranks, merged accept records + summed region
   deltas) reproduces the single-rank run exactly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, GOLDEN, bits

FIXTURES = json.load(open(os.path.join(GOLDEN, "oracle_fixtures.json")))


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _cfg(oracle_lib, **kw):
    return oracle_lib.PlannerConfig(**kw)


@pytest.mark.parametrize("case", sorted(FIXTURES["cases"]))
def test_golden_fixture(oracle_lib, obstacles, case):
    fx = FIXTURES["cases"][case]
    o = oracle_lib.Oracle(_cfg(oracle_lib, **fx["config"]), threads=4)
    o.plan(FIXTURES["initial"], FIXTURES["goal"], obstacles, fx["seed"])
    info = o.info()
    assert info["iterations"] == fx["iterations"]
    assert info["treeSize"] == fx["treeSize"]
    assert info["goalIdx"] == fx["goalIdx"]
    assert int(np.float32(info["costToGoal"]).view(np.uint32)) == fx["costToGoal_bits"]
    assert info["samples"] == fx["samples"]
    assert o.iter_logs().tolist() == fx["iter_log"]
    s, p, c = o.tree()
    for r, row in fx["rows"].items():
        r = int(r)
        assert s[r].view(np.uint32).tolist() == row["sample_bits"]
        assert int(p[r]) == row["parent"]
        assert int(c[r:r + 1].view(np.uint32)[0]) == row["cost_bits"]
    rng = o.rng()
    for i, st in fx["rng"].items():
        assert rng[int(i)].tolist() == st
    us, up = o.unexplored()
    g, gn = o.flags()
    arrays = {"samples": s, "parents": p, "costs": c, "unexplored": us, "uParent": up, "G": g, "GNew": gn,
              "rng": rng, **o.regions()}
    for k, h in fx["sha256"].items():
        assert _digest(arrays[k]) == h, k


def _demo_run(oracle_lib, obstacles, seed, **kw):
    cfg = _cfg(oracle_lib, **{**DEMO, **kw})
    o = oracle_lib.Oracle(cfg, threads=4)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    return cfg, o


@pytest.mark.parametrize("seed,fix", [(1, 0), (2, 0), (3, 1), (7, 1)])
def test_invariants_demo(oracle_lib, obstacles, seed, fix):
    cfg, o = _demo_run(oracle_lib, obstacles, seed, fixGNewClear=fix)
    info = o.info()
    n = info["treeSize"]
    s, p, c = o.tree()
    s, p, c = s[:n], p[:n], c[:n]
    # I3: topology and costs.
    assert p[0] == -1
    j = np.arange(1, n)
    assert np.all((p[1:] >= 0) & (p[1:] < j))
    assert np.array_equal(bits(c[1:]), bits((c[p[1:]] + s[1:, 6]).astype(np.float32)))
    # I4: sampled control ranges (a = 10u - 5, steering = 2*pi*u - pi, T = u + 0.05, u in (0, 1]).
    a, st, dur = s[1:, 4], s[1:, 5], s[1:, 6]
    assert np.all((a > -5.0) & (a <= 5.0))
    assert np.all((st > -np.float32(np.pi) - 1e-6) & (st <= np.float32(np.pi) + 1e-6))
    assert np.all((dur > 0.05) & (dur <= 1.05 + 1e-6))
    # I1/I2: every row replays bit-exactly from its parent and controls.  Rows inserted
    # from stale GNew flags (D6) may be invalid children; with the complete clear none.
    states, valid = oracle_lib.replay(cfg, obstacles, s[p[1:], :4], s[1:, 4:7])
    assert np.array_equal(bits(states), bits(s[1:, :4]))
    if fix:
        assert valid.all()
    else:
        assert valid.mean() > 0.9
    # I5: region counters balance.
    reg = o.regions()
    assert np.array_equal(reg["R1Valid"] + reg["R1Invalid"], reg["R1"])
    assert reg["R1"].sum() <= 1 + info["samples"]
    assert reg["R1Valid"].sum() >= n   # every row was a valid child (or the root) when drawn
    assert (reg["R2Valid"] + reg["R2Invalid"]).sum() <= reg["R1"].sum()
    avail = np.flatnonzero(reg["R2Avail"])
    assert np.all((reg["R2Valid"][avail] > 0) | (np.arange(len(reg["R2Avail"]))[avail] == _root_r2()))


def _root_r2():
    # Demo root (5, 5): R1 cell (4, 4) -> 4*16+4 = 68; R2 cell (0, 0) inside it (KGMT.cu:602-629).
    return 68 * 64


def test_goal_semantics(oracle_lib, obstacles):
    """D4: the solution is the lowest new row inside the goal radius; costToGoal its cost."""
    cfg, o = _demo_run(oracle_lib, obstacles, 1)
    info = o.info()
    s, p, c = o.tree()
    g = info["goalIdx"]
    assert g >= 0
    d = np.sqrt((s[:info["treeSize"], 0] - np.float32(2.0)) ** 2 + (s[:info["treeSize"], 1] - np.float32(18.0)) ** 2)
    inside = np.flatnonzero(d < 0.5)
    assert g == inside.min()
    assert np.float32(info["costToGoal"]) == c[g]


def test_empty_frontier_stalls(oracle_lib, obstacles):
    """D7: once G is empty an iteration is a no-op (the reference's zero-block launch);
    the loop then runs out its iteration budget with the tree unchanged."""
    cfg, o = _demo_run(oracle_lib, obstacles, 99, maxTreeSize=700, numIterations=50, goalThreshold=0.0)
    info = o.info()
    assert info["terminated"] and info["iterations"] == 50
    log = o.iter_logs()
    stalled = log[log[:, 2] == 0]
    assert len(stalled) > 0
    assert np.all(stalled[:, 5] == 0) and np.all(stalled[:, 6] == 0)          # S = A = 0
    assert np.all(stalled[:, 1] == info["treeSize"]) and np.all(stalled[:, 7] == info["treeSize"])


def test_iteration_limit(oracle_lib, obstacles):
    cfg, o = _demo_run(oracle_lib, obstacles, 5, numIterations=3, goalThreshold=0.0)
    assert o.info()["iterations"] == 3


def test_fill_batch_rule(oracle_lib, obstacles):
    """D14: with the fill rule every iteration generates floor(cap/|G|)*|G| (or cap) children."""
    cfg, o = _demo_run(oracle_lib, obstacles, 11, samplesPerIteration=4096, batchRule=1, maxTreeSize=200000,
                       numIterations=10, goalThreshold=0.0)
    for row in o.iter_logs():
        itr, before, nG, k, nExp, S, A = (int(x) for x in row[:7])
        if nG <= 4096:
            assert k == 4096 // nG and S == k * nG
        else:
            assert k == 1 and S == 4096


def _run_sharded(oracle_lib, cfg, obstacles, seed, P):
    ranks = [oracle_lib.Oracle(cfg, threads=2, nranks=P, rank=r) for r in range(P)]
    for o in ranks:
        o.begin(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    while True:
        rets = [o.expand_local() for o in ranks]
        if all(r < 0 for r in rets):
            break
        assert all(r >= 0 for r in rets)
        recs = np.concatenate([o.local_records() for o in ranks])
        deltas = np.sum([o.local_deltas() for o in ranks], axis=0).astype(np.int32)
        for o in ranks:
            o.finish(recs, deltas)
        if ranks[0].info()["terminated"]:
            break
    return ranks


@pytest.mark.parametrize("P,kw,seed", [
    (2, dict(), 1),
    (3, dict(), 2),
    (2, dict(samplesPerIteration=2048, maxTreeSize=60000, numIterations=12, goalThreshold=0.0), 4),
    (3, dict(samplesPerIteration=3000, batchRule=1, maxTreeSize=80000, numIterations=10, goalThreshold=0.0), 6),
])
def test_sharded_protocol_matches_single_rank(oracle_lib, obstacles, P, kw, seed):
    cfg = _cfg(oracle_lib, **{**DEMO, **kw})
    ref = oracle_lib.Oracle(cfg, threads=4)
    ref.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    ranks = _run_sharded(oracle_lib, cfg, obstacles, seed, P)
    rs, rp, rc = ref.tree()
    rreg = ref.regions()
    for o in ranks:
        assert o.info()["treeSize"] == ref.info()["treeSize"]
        assert o.info()["goalIdx"] == ref.info()["goalIdx"]
        assert o.iter_logs().tolist() == ref.iter_logs().tolist()
        s, p, c = o.tree()
        assert np.array_equal(bits(s), bits(rs))
        assert np.array_equal(p, rp)
        assert np.array_equal(bits(c), bits(rc))
        reg = o.regions()
        for k in rreg:
            assert np.array_equal(bits(reg[k]), bits(rreg[k])), k
