"""Uniform-grid obstacle index (include/sbmp/obstacle_grid.h):
the grid answer equals the reference's all-boxes isMotionValid
(collisionCheck.cu:6-28) for every segment, evaluated on the host through
sbmp_obstacle_grid_query and compared with a numpy brute force of the same
predicate (float32 compares, NaN compares false).  The device kernels share the
query template; tests/test_gpu_parity.py runs the planner on the grid path."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

W, H = 20.0, 20.0


def brute_free(obs, segs):
    o = obs[None, :, :]
    s = segs[:, None, :]
    with np.errstate(invalid="ignore"):
        disjoint = (s[..., 2] <= o[..., 0]) | (o[..., 2] <= s[..., 0]) | (s[..., 3] <= o[..., 1]) | \
                   (o[..., 3] <= s[..., 1])
    return disjoint.all(axis=1)


def grid_free(nat, obs, segs, g=0, w=W, h=H):
    obs = np.ascontiguousarray(obs, dtype=np.float32)
    segs = np.ascontiguousarray(segs, dtype=np.float32)
    out = np.zeros(len(segs), dtype=np.uint8)
    used = ctypes.c_int()
    nat.call("sbmp_obstacle_grid_query", obs.ctypes.data_as(ctypes.c_void_p), len(obs), w, h, g,
             segs.ctypes.data_as(ctypes.c_void_p), len(segs), out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(used))
    return out.astype(bool), used.value


def random_segments(rng, n, lo=-1.0, hi=21.0, scale=1.0):
    a = rng.uniform(lo, hi, size=(n, 2)).astype(np.float32)
    b = (a + rng.normal(0, scale, size=(n, 2))).astype(np.float32)
    return np.concatenate([np.minimum(a, b), np.maximum(a, b)], axis=1)


def c5_obstacles():
    from cudasbmp_amd import read_obstacles_csv
    return read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles_c5.csv"))


@pytest.fixture(scope="module")
def nat():
    from cudasbmp_amd import _native
    return _native


@pytest.mark.parametrize("g", [0, 1, 2, 7, 64, 256])
def test_grid_matches_brute_force_on_c5(nat, g):
    obs = c5_obstacles()
    rng = np.random.default_rng(5 + g)
    segs = np.concatenate([random_segments(rng, 4000, scale=0.2), random_segments(rng, 500, scale=3.0)])
    got, used = grid_free(nat, obs, segs, g)
    assert used == (g if g > 0 else used) and used >= 1
    want = brute_free(obs, segs)
    assert np.array_equal(got, want)
    assert 0.05 < want.mean() < 0.99   # both outcomes are exercised


def test_grid_edge_cases(nat):
    rng = np.random.default_rng(11)
    g = 8
    cell = W / g
    edges = np.arange(0, g + 1, dtype=np.float32) * np.float32(cell)
    obs = [
        [e0, e1, e0 + cell, e1 + cell] for e0, e1 in zip(edges[:-1], edges[1:])   # boxes exactly on cell lines
    ] + [
        [-5.0, -5.0, -1.0, -1.0],       # outside the workspace
        [25.0, 3.0, 30.0, 4.0],
        [6.0, 6.0, 4.0, 8.0],           # inverted in x
        [np.nan, 2.0, 3.0, 3.0],        # NaN coordinate: listed everywhere
        [-np.inf, 10.0, np.inf, 10.5],  # infinite extent
        [7.5, 7.5, 7.5, 7.5],           # degenerate
    ]
    obs = np.array(obs, dtype=np.float32)
    segs = [random_segments(rng, 3000, lo=-6.0, hi=32.0, scale=2.0)]
    pts = rng.choice(edges, size=(2000, 2)).astype(np.float32)   # segments touching cell lines exactly
    d = rng.choice(np.array([0.0, cell, 2 * cell, 0.01], dtype=np.float32), size=(2000, 2))
    segs.append(np.concatenate([pts, pts + d], axis=1))
    segs.append(np.array([[4.5, 6.5, 5.5, 7.0], [-10, -10, 40, 40], [7.5, 7.5, 7.5, 7.5], [7.4, 7.4, 7.6, 7.6]],
                         dtype=np.float32))
    segs = np.concatenate(segs)
    got, used = grid_free(nat, obs, segs, g)
    assert used == g
    assert np.array_equal(got, brute_free(obs, segs))


def test_grid_empty_and_small(nat):
    rng = np.random.default_rng(3)
    segs = random_segments(rng, 100)
    got, _ = grid_free(nat, np.zeros((0, 4), np.float32), segs)
    assert got.all()
    obs = np.array([[2, 2, 4, 4]], dtype=np.float32)
    got, used = grid_free(nat, obs, segs)
    assert used == 1 and np.array_equal(got, brute_free(obs, segs))


def test_grid_caps_copies_of_huge_boxes(nat):
    # every box covers the workspace: the builder lowers the resolution instead of
    # copying each box into every one of 256 x 256 cells
    obs = np.tile(np.array([[-1, -1, 21, 21]], dtype=np.float32), (600, 1))
    rng = np.random.default_rng(4)
    segs = random_segments(rng, 50)
    got, used = grid_free(nat, obs, segs, 256)
    assert used * used * 600 <= (1 << 25)
    assert np.array_equal(got, brute_free(obs, segs))
