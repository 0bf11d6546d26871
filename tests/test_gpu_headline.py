"""GPU parity at the benchmark configurations (BASELINE.json configs c1-c5), whole state
bit-exact against the CPU oracle -- not properties.

  c1  exactly as systems/c1.yaml states it: the R2 point agent, 1,024 samples per
      iteration, M = 2^20, fill rule, complete GNew clear, 100 iterations, read through
      the library's config parser (sbmp_load_system_config).

  c3  the exact bench mode: car, S = 262,144/iteration, M = 2^24, fill rule (D14),
      complete GNew clear, seed 20240807, 72 iterations: covers the driver's timed
      window (iterations 6-25 of `bench.py --warmup 5 --steps 20`) and bench.py's own
      default window (21-70), including the steady state where the planner workgroup
      inserts (A <= kPlannerInsertMax) and the R2 key-log folds at 32 and 64.
  c3r the same with the reference's partial GNew clear (D6), 40 iterations.
  c2  the R2 point agent at 262,144 samples/iteration.
  c4  1,048,576 samples/iteration: on one rank (more blocks than one launch holds)
      and as an 8-rank local shard group on one GPU (the sharded data flow of
      DESIGN.md §7 with the all-reduce replaced by a sum kernel), M = 2^25 as bench.py
      uses for more than 2 ranks.
  c5  the 10,000-box field at 1,048,576 samples/iteration (uniform-grid index).
Reference: KGMT.cu:118-292 (loop), 151-249 (batch, insertion); DESIGN.md D6/D14.
"""
import os

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, ROOT
from test_gpu_parity import _oracle, assert_same_state

pytestmark = pytest.mark.gpu

BENCH_SEED = 20240807


def _run(kw, seed, obs, P=0, threads=16):
    from cudasbmp_amd import KGMT, DeviceBuffer
    cfg = dict(DEMO)
    extra = {k: kw[k] for k in ("samplesPerIteration", "agent", "fixGNewClear", "batchRule") if k in kw}
    cfg.update({k: v for k, v in kw.items() if k not in extra})
    g = KGMT(**cfg, **extra, _local_group=P)
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, DeviceBuffer(obs), len(obs), seed=seed)
    o = _oracle(cfg, extra, threads=threads)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obs, seed)
    return g, o, r


def _bench_kw(S, iters, **kw):
    d = dict(samplesPerIteration=S, maxTreeSize=1 << 24, numIterations=iters, goalThreshold=0.0, batchRule="fill",
             fixGNewClear=True)
    d.update(kw)
    return d


def _c5_obstacles():
    from cudasbmp_amd import read_obstacles_csv
    return read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles_c5.csv"))


def test_c1_as_configured_bit_exact(oracle_lib):
    from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv
    from cudasbmp_amd.config import workload
    cfg = workload("c1")
    assert cfg["agent"] == "point" and cfg["samplesPerIteration"] == 1024 and cfg["batchRule"] == "fill"
    obs = read_obstacles_csv(cfg["obstacles"])
    pl = dict(cfg["planner"])
    extra = dict(samplesPerIteration=1024, agent="point", batchRule="fill", fixGNewClear=True)
    g = KGMT(**pl, **extra)
    r = g.plan(cfg["initial"], cfg["goal"], DeviceBuffer(obs), len(obs), seed=BENCH_SEED)
    o = _oracle(pl, extra)
    o.plan(cfg["initial"], cfg["goal"], obs, BENCH_SEED)
    assert r.iterations == pl["numIterations"] == 100
    assert g.iter_log()[:, 5].max() == 1024   # fill rule: S = k * nExp <= 1024 (D14)
    assert_same_state(g, o, label="c1 as configured")


def test_c3_bench_mode_bit_exact(obstacles, oracle_lib):
    g, o, r = _run(_bench_kw(262144, 72), BENCH_SEED, obstacles)
    info = g.path_info()
    assert info["form"] == "k_step", info
    log = g.iter_log()
    assert r.iterations == 72 and log[5:, 5].min() > 250000
    assert (log[20:, 6] <= 4096).all(), "steady state: the planner workgroup inserts"
    assert_same_state(g, o, label="c3 bench mode")


def test_c3_reference_clear_bit_exact(obstacles, oracle_lib):
    g, o, r = _run(_bench_kw(262144, 40, fixGNewClear=False), BENCH_SEED, obstacles)
    assert r.iterations == 40
    assert_same_state(g, o, label="c3 reference clear")


def test_c2_point_bit_exact(obstacles, oracle_lib):
    g, o, r = _run(_bench_kw(262144, 30, agent="point"), BENCH_SEED, obstacles)
    assert r.iterations == 30 and g.iter_log()[:, 5].min() > 200000
    assert_same_state(g, o, label="c2 point")


def test_c4_one_rank_1M_bit_exact(obstacles, oracle_lib):
    g, o, r = _run(_bench_kw(1 << 20, 5, maxTreeSize=1 << 25), BENCH_SEED, obstacles)
    assert g.iter_log()[:, 5].max() == 1 << 20
    assert_same_state(g, o, label="c4 one rank")


def test_c4_local_group_8_ranks_1M_bit_exact(obstacles, oracle_lib):
    g, o, r = _run(_bench_kw(1 << 20, 5, maxTreeSize=1 << 25), BENCH_SEED, obstacles, P=8)
    assert g.iter_log()[:, 5].max() == 1 << 20
    assert_same_state(g, o, label="c4 8-rank local group")


@pytest.mark.parametrize("blocks,clear", [(1031, True), (2049, False)])
def test_two_launch_grouped_inserts_ragged_bit_exact(blocks, clear, obstacles, oracle_lib):
    """Above 1,024 blocks k_finish's insert workgroups take up to 4 blocks each at a
    stride of the group count (insert_blocks): 1,031 blocks (264 groups, the last blocks
    of the stride past the end) and 2,049 blocks (520 groups) with the reference's
    partial GNew clear (D6), whole state bit-exact."""
    g, o, r = _run(_bench_kw(256 * blocks, 6, maxTreeSize=1 << 23, fixGNewClear=clear), BENCH_SEED, obstacles)
    info = g.path_info()
    assert info["form"] == "two-launch", info
    assert g.iter_log()[:, 5].max() == 256 * blocks
    assert_same_state(g, o, label=f"two-launch, {blocks} blocks")


def test_c5_1M_bit_exact(oracle_lib):
    obs = _c5_obstacles()
    assert len(obs) == 10000
    g, o, r = _run(_bench_kw(1 << 20, 3), BENCH_SEED, obs)
    assert g.iter_log()[:, 5].max() == 1 << 20
    assert_same_state(g, o, label="c5 1M")


def test_c3_lds_2048_boxes_takes_the_two_launch_form(oracle_lib):
    """k_step needs all 1 + 1,024 workgroups resident (its expanders wait for workgroup
    0); a 2,048-box LDS list (32 KB per workgroup) leaves 4 per CU, 1,024 on the chip,
    so begin() picks the two-launch form (KGMT.cu:151-249 as k_expand + k_finish).
    Bit-exact against the oracle at c3 size."""
    obs = _c5_obstacles()[:2048].copy()
    g, o, r = _run(_bench_kw(262144, 3), BENCH_SEED, obs)
    info = g.path_info()
    assert info["obstacle_form"] == "lds" and info["form"] == "two-launch", info
    assert 0 < info["resident_groups"] < info["needed_groups"] == 1025, info
    assert g.iter_log()[:, 5].max() == 262144
    assert_same_state(g, o, label="c3 2,048-box LDS list")


def test_sharded_lds_2048_boxes_takes_the_grid(oracle_lib):
    """A sharded rank keeps k_step (its exchange layout), so when the LDS list does not
    leave room for all its workgroups it indexes the boxes with the uniform grid: 2 ranks
    of 1,024 blocks each (524,288 children), bit-exact."""
    obs = _c5_obstacles()[:2048].copy()
    g, o, r = _run(_bench_kw(1 << 19, 2, maxTreeSize=1 << 25), BENCH_SEED, obs, P=2)
    info = g.path_info()
    assert info["form"] == "k_step" and info["obstacle_form"] == "grid", info
    assert info["needed_groups"] == 1025 and info["resident_groups"] >= 1025, info
    assert_same_state(g, o, label="2 ranks, 2,048-box list on the grid")


def test_c3_path_info_is_k_step():
    from cudasbmp_amd import KGMT, DeviceBuffer
    from conftest import OBSTACLES_CSV
    obs = np.loadtxt(OBSTACLES_CSV, delimiter=",", dtype=np.float32).reshape(-1, 4)
    cfg = dict(DEMO)
    kw = _bench_kw(262144, 2)
    extra = {k: kw.pop(k) for k in ("samplesPerIteration", "fixGNewClear", "batchRule")}
    cfg.update(kw)
    g = KGMT(**cfg, **extra)
    g.plan(DEMO_INITIAL, DEMO_GOAL, DeviceBuffer(obs), len(obs), seed=BENCH_SEED)
    info = g.path_info()
    assert info["form"] == "k_step" and info["obstacle_form"] == "registers" and info["exchange"] == "none", info
    assert info["resident_groups"] >= info["needed_groups"] == 1025, info


@pytest.mark.parametrize("P", [2, 8])
def test_c5_sharded_per_rank_shape_bit_exact(P, oracle_lib):
    """The kernel every rank of the 8-GPU c5 configuration runs (BASELINE.json c5: 1,048,576
    children per iteration over 8 GPUs = 131,072 per rank on the 10,000-box field): the
    sharded k_step with the uniform-grid obstacle index, here as a local shard group of P
    ranks of 131,072 children each on one GPU, 6 iterations, whole state bit-exact.
    Reference: collisionCheck.cu:16-28 (the per-step box loop), KGMT.cu:341-414."""
    obs = _c5_obstacles()
    g, o, r = _run(_bench_kw(131072 * P, 6, maxTreeSize=1 << 25), BENCH_SEED, obs, P=P)
    info = g.path_info()
    assert info["form"] == "k_step" and info["obstacle_form"] == "grid" and info["nranks"] == P, info
    assert info["needed_groups"] == 1 + 512 and info["resident_groups"] >= info["needed_groups"], info
    assert info["row_table_lds"], info
    assert r.iterations == 6 and g.iter_log()[:, 5].max() == 131072 * P
    assert_same_state(g, o, label=f"c5 per-rank shape, {P} ranks")


def test_c5_sharded_1024_rows_without_row_table(oracle_lib):
    """8 sharded ranks of 262,144 children (1,024 rows each) on the 10,000-box field: the
    grid's cell-start table (20 KB) and the u16 row table of 8,192 blocks (16 KB) in LDS
    leave three workgroups per CU (768 of the 1,025 k_step needs; ADVICE r05: begin()
    refused this shape in round 5), so begin() drops the row table (row positions from the
    exchange's block words, one more L2 round trip) and keeps k_step on the grid.  A local
    group of 8 ranks on one GPU, 3 iterations, whole state bit-exact."""
    obs = _c5_obstacles()
    g, o, r = _run(_bench_kw(262144 * 8, 3, maxTreeSize=1 << 25), BENCH_SEED, obs, P=8)
    info = g.path_info()
    assert info["form"] == "k_step" and info["obstacle_form"] == "grid" and info["nranks"] == 8, info
    assert info["needed_groups"] == 1 + 1024 and info["resident_groups"] >= info["needed_groups"], info
    assert not info["row_table_lds"], info
    assert r.iterations == 3 and g.iter_log()[:, 5].max() == 262144 * 8
    assert_same_state(g, o, label="c5 1,024 rows per rank, no row table")


@pytest.mark.parametrize("P", [2, 8])
def test_sharded_row_table_off_bit_exact(P, obstacles, oracle_lib, monkeypatch):
    """SBMP_C16_LDS=0 forces the block-word form of row positions on the c3 workload:
    every lookup (parents from t-1's lists, the expanders' own-row inserts, the planner's
    inserts) reads the row's block words; whole state bit-exact."""
    monkeypatch.setenv("SBMP_C16_LDS", "0")
    g, o, r = _run(_bench_kw(16384 * P, 12, maxTreeSize=1 << 22), BENCH_SEED, obstacles, P=P)
    info = g.path_info()
    assert info["form"] == "k_step" and not info["row_table_lds"], info
    assert_same_state(g, o, label=f"row table off, {P} ranks")
