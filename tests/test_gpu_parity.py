"""GPU parity: the HIP planner (through the C ABI) against the CPU oracle.

Bar (north star): bit-exact node indices, accept masks and tree arrays; states
compared bit-exactly too (the 1e-5 tolerance is not needed: both sides run the
same float operation sequence).
"""
import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, bits

pytestmark = pytest.mark.gpu


def _mk(**kw):
    from cudasbmp_amd import KGMT
    cfg = dict(DEMO)
    extra = {k: kw.pop(k) for k in ("samplesPerIteration", "agent", "fixGNewClear", "batchRule") if k in kw}
    cfg.update(kw)
    return KGMT(**cfg, **extra), cfg, extra


def _oracle(cfg, extra, threads=8):
    from oracle.pyoracle import Oracle, PlannerConfig
    pc = PlannerConfig(**cfg, samplesPerIteration=extra.get("samplesPerIteration", 0),
                       agent=1 if extra.get("agent", "car") == "point" else 0,
                       fixGNewClear=int(extra.get("fixGNewClear", 0)),
                       batchRule=1 if extra.get("batchRule", "reference") == "fill" else 0)
    return Oracle(pc, threads=threads)


def _first_diff(a, b):
    a, b = bits(a), bits(b)
    d = np.nonzero((a != b).reshape(len(a), -1).any(axis=1))[0]
    return int(d[0]) if len(d) else -1


def assert_same_state(g, o, check_unexplored=True, label=""):
    lg, lo = g.iter_log(), o.iter_logs()
    assert lg.shape == lo.shape and np.array_equal(lg, lo), f"{label} iteration logs differ:\n{lg}\n{lo}"
    sg, pg, cg = g.tree()
    so, po, co = o.tree()
    assert np.array_equal(pg, po), f"{label} parents differ at row {_first_diff(pg, po)}"
    assert np.array_equal(bits(sg), bits(so)), f"{label} tree samples differ at row {_first_diff(sg, so)}"
    assert np.array_equal(bits(cg), bits(co)), f"{label} costs differ at row {_first_diff(cg, co)}"
    Gg, GNg = g.flags()
    Go, GNo = o.flags()
    assert np.array_equal(Gg, Go), f"{label} G differs at {_first_diff(Gg, Go)}"
    assert np.array_equal(GNg, GNo), f"{label} GNew (accept mask) differs at {_first_diff(GNg, GNo)}"
    rg, ro = g.regions(), o.regions()
    for k in ro:
        assert np.array_equal(bits(rg[k]), bits(ro[k])), f"{label} {k} differs at {_first_diff(rg[k], ro[k])}"
    if check_unexplored:
        ug, upg = g.unexplored()
        uo, upo = o.unexplored()
        assert np.array_equal(upg, upo), f"{label} uParentIdx differs at {_first_diff(upg, upo)}"
        assert np.array_equal(bits(ug), bits(uo)), f"{label} unexplored differs at {_first_diff(ug, uo)}"
    assert np.array_equal(g.rng(), o.rng()), f"{label} RNG states differ"
    info = o.info()
    r = g.result()
    assert r.iterations == info["iterations"]
    assert r.treeSize == info["treeSize"]
    assert r.goalIndex == info["goalIdx"]
    assert bits(np.float32(r.costToGoal)) == bits(np.float32(info["costToGoal"]))


@pytest.fixture(scope="module")
def d_obs(obstacles):
    from cudasbmp_amd import DeviceBuffer
    return DeviceBuffer(obstacles)


def test_rng_init_matches_oracle(d_obs, obstacles, oracle_lib):
    g, cfg, extra = _mk(maxTreeSize=5000)
    o = _oracle(cfg, extra)
    for seed in (0, 1, 0xFFFFFFFFFFFFFFFF, 1723000000):
        g.begin(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed)
        o.begin(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
        assert np.array_equal(g.rng(), o.rng()), f"seed {seed}"


@pytest.mark.parametrize("seed", [1, 2, 3, 7, 12345, 1723000000])
def test_demo_plan_bit_exact(seed, d_obs, obstacles, oracle_lib):
    """Full KGMT::plan on the reference demo (main.cu:19-46): whole state bit-exact."""
    g, cfg, extra = _mk()
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=seed)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    assert r.iterations > 1
    assert_same_state(g, o, label=f"seed {seed}")


def test_stepwise_bit_exact(d_obs, obstacles, oracle_lib):
    g, cfg, extra = _mk()
    o = _oracle(cfg, extra)
    g.begin(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), 42)
    o.begin(DEMO_INITIAL, DEMO_GOAL, obstacles, 42)
    for it in range(1, 8):
        a = g.step(1)
        b = o.step()
        assert b
        assert_same_state(g, o, label=f"iteration {it}")
        if not a:
            break


@pytest.mark.parametrize("kw", [
    dict(samplesPerIteration=4096, maxTreeSize=200000, numIterations=15, goalThreshold=0.0),
    dict(samplesPerIteration=1000, maxTreeSize=50000, numIterations=20),
    dict(agent="point"),
    dict(agent="point", samplesPerIteration=2048, maxTreeSize=100000, numIterations=12, goalThreshold=0.0),
    dict(fixGNewClear=True),
    dict(maxTreeSize=700, numIterations=50),            # V2 branch, k < 32, tree-full termination (D13)
    dict(maxTreeSize=64, numIterations=50),             # tiny capacity: k = 0 path
    dict(n=4),                                          # different R2 sub-grid
    dict(n=16, maxTreeSize=20000),                      # > kLogMaxR2 cells: direct R2 atomics
    dict(n=11, maxTreeSize=20000),                      # largest key-log grid (121 KB fold histogram)
    dict(numDisc=1),
    dict(numDisc=25, agentLength=2.5),
    dict(numDisc=7, agentLength=1.3),                   # reciprocal-multiply division (host-verified divisors)
    dict(n=3, numDisc=13, agentLength=0.7),
    dict(agentLength=3e-7, numIterations=5),            # L below 2^-20: no reciprocal, IEEE division of v / L
    dict(samplesPerIteration=8192, batchRule="fill", maxTreeSize=300000, numIterations=12, goalThreshold=0.0),
    dict(samplesPerIteration=3000, batchRule="fill", maxTreeSize=40000, numIterations=40),   # fills the tree
    dict(samplesPerIteration=4096, batchRule="fill", agent="point", maxTreeSize=100000, numIterations=10),
    dict(numIterations=0),
    dict(numIterations=1),
    dict(goalThreshold=0.0, numIterations=30),
])
def test_configs_bit_exact(kw, d_obs, obstacles, oracle_lib):
    g, cfg, extra = _mk(**dict(kw))
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=99)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, 99)
    assert_same_state(g, o, label=str(kw))


@pytest.mark.parametrize("case", ["no_obstacles", "root_outside", "root_in_obstacle_row", "many_obstacles",
                                  "dense_obstacles_global_path", "goal_near_root", "one_obstacle",
                                  "eight_obstacles_registers", "nine_obstacles_lds"])
def test_edge_cases_bit_exact(case, obstacles, oracle_lib):
    from cudasbmp_amd import DeviceBuffer
    init, goal, obs = list(DEMO_INITIAL), list(DEMO_GOAL), obstacles
    if case == "no_obstacles":
        obs = np.zeros((0, 4), dtype=np.float32)
    elif case == "root_outside":
        init[0] = -1.0          # r1 = -1: root seeds skipped (D3); every child invalid -> stall (D7)
    elif case == "root_in_obstacle_row":
        init[1] = 7.0           # root inside the (0,6)-(18,8) wall
    elif case in ("many_obstacles", "dense_obstacles_global_path"):
        rng = np.random.default_rng(20240807)
        n = 600 if case == "many_obstacles" else 3000   # > 2048: obstacles read from global memory
        c = rng.uniform(0, 20, size=(n, 2)).astype(np.float32)
        c = c[np.hypot(c[:, 0] - 5, c[:, 1] - 5) > 0.5]
        h = rng.uniform(0.02, 0.08, size=(len(c), 2)).astype(np.float32)
        obs = np.concatenate([c - h, c + h], axis=1).astype(np.float32)
    elif case == "goal_near_root":
        goal[0], goal[1] = 5.2, 5.1
    elif case == "one_obstacle":
        obs = obstacles[4:5]
    elif case in ("eight_obstacles_registers", "nine_obstacles_lds"):   # kMaxRegObs = 8
        extra_boxes = np.array([[10, 12, 11, 13], [14, 3, 15, 4], [12, 15, 13, 16], [16, 10, 17, 11]],
                               dtype=np.float32)
        obs = np.concatenate([obstacles, extra_boxes[:3 if case.startswith("eight") else 4]])
    g, cfg, extra = _mk(numIterations=40)
    d = DeviceBuffer(obs) if len(obs) else None
    g.plan(init, goal, d, len(obs), seed=5)
    o = _oracle(cfg, extra)
    o.plan(init, goal, obs, 5)
    assert_same_state(g, o, label=case)


def test_full_size_first_iterations_bit_exact(d_obs, obstacles, oracle_lib):
    """Bench configuration (c3: car, S=262144/iter, M=2^24): first iterations bit-exact."""
    g, cfg, extra = _mk(samplesPerIteration=262144, maxTreeSize=1 << 24, numIterations=4, goalThreshold=0.0,
                        batchRule="fill")
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=2024)
    o = _oracle(cfg, extra, threads=16)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, 2024)
    assert g.iter_log()[:, 5].min() > 250000
    assert_same_state(g, o, check_unexplored=True, label="full-size")


@pytest.mark.parametrize("fix_clear", [False, True])
def test_full_size_properties(fix_clear, d_obs, obstacles, oracle_lib):
    """Size-independent invariants of the reference's semantics on a long bench-size run:
    I1 replay (re-propagating parent + stored controls reproduces every node bit-exactly;
    the replay is also collision-free for every node when the GNew clear is complete --
    with the reference's partial clear (D6) a stale accept flag re-inserts whatever child
    last used that slot, valid or not), I3 parent < row and cost = cost[parent] + duration
    (bitwise), I4 control ranges, I5 region-count conservation."""
    from oracle.pyoracle import PlannerConfig, replay
    M = 1 << 24
    g, cfg, extra = _mk(samplesPerIteration=262144, maxTreeSize=M, numIterations=40, goalThreshold=0.0,
                        batchRule="fill", fixGNewClear=fix_clear)
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=77)
    assert r.iterations == 40
    n = min(r.treeSize, M)
    assert n > 10000
    s, p, c = g.tree()
    s, p, c = s[:n], p[:n], c[:n]
    assert p[0] == -1 and np.all(p[1:] >= 0) and np.all(p[1:] < np.arange(1, n))
    exp_cost = (c[p[1:]] + s[1:, 6]).astype(np.float32)
    assert np.array_equal(bits(exp_cost), bits(c[1:]))
    a, st, du = s[1:, 4], s[1:, 5], s[1:, 6]
    assert np.all((a > -5) & (a <= 5)) and np.all((st >= -np.pi) & (st <= np.pi))
    assert np.all((du > 0.05) & (du <= 1.0500001))
    pc = PlannerConfig(**cfg, samplesPerIteration=262144, batchRule=1)
    out, valid = replay(pc, obstacles, s[p[1:], :4], s[1:, 4:7], threads=16)
    assert np.array_equal(bits(out), bits(s[1:, :4])), "replayed states differ"
    if fix_clear:
        assert valid.all(), f"{(~valid).sum()} inserted nodes collide or leave the workspace"
    else:
        assert valid.mean() > 0.5
    # I5: R1Valid + R1Invalid = R1; every cell with a valid child is available.
    reg = g.regions()
    assert np.array_equal(reg["R1Valid"] + reg["R1Invalid"], reg["R1"])
    assert int(reg["R1"].sum()) <= r.samplesGenerated + 1
    assert np.all(reg["R2Avail"][reg["R2Valid"] > 0] == 1)


@pytest.mark.parametrize("P,kw,seed", [
    (2, dict(), 1),
    (3, dict(), 2),
    (4, dict(fixGNewClear=True), 3),
    (2, dict(samplesPerIteration=4096, maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 99),
    (8, dict(samplesPerIteration=8192, batchRule="fill", maxTreeSize=300000, numIterations=12, goalThreshold=0.0), 7),
    (3, dict(maxTreeSize=700, numIterations=50), 99),
    (2, dict(agent="point", samplesPerIteration=2048, maxTreeSize=100000, numIterations=12, goalThreshold=0.0), 5),
])
def test_local_shard_group_bit_exact(P, kw, seed, d_obs, obstacles, oracle_lib):
    """The sharded data flow (owned slots, one k_step per rank and iteration, the
    owners' lists read through the record buffers, the summed exchange buffer, every
    rank inserting its row of blocks) with P ranks on one GPU equals the oracle."""
    from cudasbmp_amd import KGMT
    cfg = dict(DEMO)
    extra = {k: kw[k] for k in ("samplesPerIteration", "agent", "fixGNewClear", "batchRule") if k in kw}
    cfg.update({k: v for k, v in kw.items() if k not in extra})
    g = KGMT(**cfg, **extra, _local_group=P)
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=seed)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    assert_same_state(g, o, label=f"P={P} {kw}")


@pytest.mark.parametrize("P,seed", [(2, 1), (4, 2)])
def test_local_shard_group_k_step_goal(P, seed, d_obs, obstacles, oracle_lib):
    """Sharded ranks take k_step (no k_expand / k_pack / k_finish launch), and the goal
    found through the exchanged row and block words stops the run where the oracle's does."""
    from cudasbmp_amd import KGMT
    cfg = dict(DEMO)
    g = KGMT(**cfg, _local_group=P)
    g.set_profiling(True)
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=seed)
    stats = g.kernel_stats()
    assert stats["k_step"][0] > 0
    assert all(stats.get(k, (0, 0.0))[0] == 0 for k in ("k_expand", "k_pack", "k_finish"))
    assert r.goalIndex >= 0, "demo seeds solve"
    o = _oracle(cfg, {})
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    assert_same_state(g, o, label=f"P={P} goal")


def test_rccl_single_rank_sharded_path(d_obs, obstacles, oracle_lib):
    """The RCCL rank path end to end on one GPU: ncclCommInitRank, the fused
    ncclAllReduce per iteration, the IPC record-buffer exchange (own buffer) and
    the R2 counter all-reduce at export, with k_step reading the lists through it."""
    import ctypes
    from cudasbmp_amd import KGMT
    from cudasbmp_amd import _native as nat
    uid = (ctypes.c_uint8 * nat.SBMP_COMM_ID_BYTES)()
    nat.call("sbmp_comm_get_unique_id", uid)
    kw = dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=20, goalThreshold=0.0)
    cfg = dict(DEMO)
    extra = {k: kw[k] for k in ("samplesPerIteration", "batchRule")}
    cfg.update({k: v for k, v in kw.items() if k not in extra})
    g = KGMT(**cfg, **extra, _sharded=(bytes(uid), 1, 0))
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=21)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, 21)
    assert_same_state(g, o, label="rccl single rank")


def _c5_obstacles():
    import os
    from conftest import ROOT
    from cudasbmp_amd import read_obstacles_csv
    return read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles_c5.csv"))


@pytest.mark.parametrize("agent", ["car", "point"])
@pytest.mark.parametrize("case,variant", [("demo_boxes_grid", "4"), ("random600_grid", "4"), ("c5_auto", "0"),
                                          ("c5_global_list", "5")])
def test_obstacle_grid_bit_exact(case, variant, agent, obstacles, oracle_lib, monkeypatch):
    """The uniform-grid obstacle index (default above kMaxLdsObs boxes,
    forced by SBMP_EXPAND_VARIANT=4) and the global all-boxes loop (variant 5) against
    the oracle's isMotionValid loop (collisionCheck.cu:16-28)."""
    from cudasbmp_amd import DeviceBuffer
    monkeypatch.setenv("SBMP_EXPAND_VARIANT", variant)
    if case == "demo_boxes_grid":
        obs, kw = obstacles, dict(numIterations=40)
    elif case == "random600_grid":
        rng = np.random.default_rng(7)
        c = rng.uniform(-1, 21, size=(600, 2)).astype(np.float32)
        h = rng.uniform(0.02, 0.3, size=(600, 2)).astype(np.float32)
        obs = np.concatenate([c - h, c + h], axis=1).astype(np.float32)
        obs = obs[np.hypot(c[:, 0] - 5, c[:, 1] - 5) > 0.8]
        kw = dict(numIterations=40)
    else:   # the c5 field: 10,000 boxes, grid chosen automatically (or the global loop)
        obs = _c5_obstacles()
        kw = dict(numIterations=12, samplesPerIteration=8192, batchRule="fill", goalThreshold=0.0)
    g, cfg, extra = _mk(agent=agent, **kw)
    g.plan(DEMO_INITIAL, DEMO_GOAL, DeviceBuffer(obs), len(obs), seed=31)
    o = _oracle(cfg, extra, threads=16)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obs, 31)
    assert g.result().iterations > 3
    assert_same_state(g, o, label=f"{case} {agent}")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_solution_path(seed, d_obs, obstacles, oracle_lib):
    """Solution extraction: the path root .. goal node equals the
    oracle tree's parent chain; it starts at the root, ends inside the goal radius
    and every cost is its parent's cost plus its duration (KGMT.cu:631-633)."""
    g, cfg, extra = _mk()
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=seed)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    s, p, c = o.tree()
    assert r.goalIndex >= 0, "demo seeds 1-3 solve"
    want = [r.goalIndex]
    while p[want[-1]] >= 0:
        want.append(int(p[want[-1]]))
    want = want[::-1]
    rows, samples, costs = g.solution_path()
    assert rows.tolist() == want and rows[0] == 0
    assert np.array_equal(bits(samples), bits(s[rows])) and np.array_equal(bits(costs), bits(c[rows]))
    assert np.hypot(samples[-1, 0] - DEMO_GOAL[0], samples[-1, 1] - DEMO_GOAL[1]) < cfg["goalThreshold"]
    assert np.array_equal(bits(costs[1:]), bits((costs[:-1] + samples[1:, 6]).astype(np.float32)))
    assert bits(np.float32(costs[-1])) == bits(np.float32(r.costToGoal))
    mid = int(rows[len(rows) // 2])   # any row: its own chain
    r2, _, _ = g.solution_path(mid)
    assert r2.tolist() == want[:len(want) // 2 + 1]
    with pytest.raises(RuntimeError):
        g.solution_path(r.treeSize + 5)


def test_solution_path_without_solution(d_obs, obstacles):
    g, cfg, extra = _mk(numIterations=2)
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=4)
    assert r.goalIndex == -1
    rows, samples, costs = g.solution_path()
    assert len(rows) == 0 and samples.shape == (0, 7)
    rows, _, _ = g.solution_path(0)
    assert rows.tolist() == [0]


@pytest.mark.parametrize("kw", [dict(), dict(fixGNewClear=True), dict(agent="point"),
                                dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=100000,
                                     numIterations=12, goalThreshold=0.0)])
def test_two_kernel_form_bit_exact(kw, d_obs, obstacles, oracle_lib, monkeypatch):
    """The two-launch form (k_expand + k_finish; sharded ranks and more than
    kMaxStepBlocks blocks use it) forced on a single rank with SBMP_STEP=0."""
    monkeypatch.setenv("SBMP_STEP", "0")
    g, cfg, extra = _mk(**kw)
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=17)
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, 17)
    assert_same_state(g, o, label=f"two-kernel {kw}")


def test_more_blocks_than_the_step_kernel_holds(d_obs, obstacles, oracle_lib):
    """300,000 slots = 1,172 blocks > kMaxStepBlocks: the planner falls back to the
    two-launch form on its own."""
    g, cfg, extra = _mk(samplesPerIteration=300000, maxTreeSize=700000, numIterations=3, goalThreshold=0.0,
                        batchRule="fill")
    g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=8)
    o = _oracle(cfg, extra, threads=16)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, 8)
    assert g.iter_log()[:, 5].max() > 262144
    assert_same_state(g, o, label="1172 blocks")

