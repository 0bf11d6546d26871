"""Legacy random-tree generators of the reference's Planner interface (SURVEY.md §8f-4;
include/planners/Planner.cuh:6-12, src/planners/NaivePlanner.cu, CostPropPlanner.cu —
not built by the reference's CMake).  The oracle restates both kernels
(oracle/kgmt_oracle.cpp oracle_random_tree); the reference itself cannot be run here
(CUDA), so this oracle is parity-unpinned beyond the XORWOW and sin/cos/tan pins it
shares with the KGMT oracle.  GPU tests: sbmp_random_tree bit-exact against it."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, bits

ROOT_STATE = (5.0, 5.0, 0.0, 1.0, 0.0, 0.0, 0.0)


def test_oracle_generators_structure(oracle_lib):
    from oracle.pyoracle import random_tree
    cp = random_tree("costprop", ROOT_STATE, 3, 4, 32)
    nv = random_tree("naive", ROOT_STATE, 3, 4, 32)
    assert cp.shape == nv.shape == (3, 128, 7)
    assert np.array_equal(bits(cp[0, 0]), bits(nv[0, 0]))      # both seed sample 0 with curand_init(0, 0, 0)
    for t in (cp, nv):
        a, st, dur = t[..., 4], t[..., 5], t[..., 6]
        assert np.all((a >= -2.5) & (a <= 2.5)) and np.all(np.abs(st) <= np.pi / 2 + 1e-6)
        assert np.all((dur >= 0) & (dur <= 0.3))
        assert len(np.unique(t[..., 4])) > 100                  # independent draws
    # naive seeds each sample by its output index: row 0 does not depend on the row count
    # (costprop seeds by gtid * rows, CostPropPlanner.cu:69, so it does)
    one = random_tree("naive", ROOT_STATE, 1, 4, 32)
    assert np.array_equal(bits(one[0]), bits(nv[0]))
    assert not np.array_equal(bits(random_tree("costprop", ROOT_STATE, 1, 4, 32)[0]), bits(cp[0]))


def test_legacy_demo_compiles():
    lib = os.path.join(ROOT, "cudasbmp_amd", "libsbmp.so")
    if not os.path.exists(lib):
        pytest.skip("libsbmp.so not built")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "demos"), "random_tree"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    nm = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(ROOT, "demos", "random_tree")],
                        capture_output=True, text=True).stdout
    assert "sbmp_random_tree" in nm


@pytest.mark.gpu
@pytest.mark.parametrize("kind,rows,blocks,tpb", [("naive", 0, 0, 0), ("costprop", 0, 0, 0), ("costprop", 4, 6, 64),
                                                   ("naive", 3, 5, 96)])
def test_random_tree_bit_exact(kind, rows, blocks, tpb, oracle_lib):
    from cudasbmp_amd import random_tree
    from oracle.pyoracle import random_tree as oracle_tree
    g, ms = random_tree(kind, ROOT_STATE, rows, blocks, tpb)
    R, B, T = g.shape[0], blocks or (32 if kind == "naive" else 512), tpb or (32 if kind == "naive" else 1024)
    assert g.shape == (R, B * T, 7) and ms > 0
    o = oracle_tree(kind, ROOT_STATE, R, B, T)
    assert np.array_equal(bits(g), bits(o))


@pytest.mark.gpu
def test_legacy_demo_runs(tmp_path, oracle_lib):
    from oracle.pyoracle import random_tree as oracle_tree
    test_legacy_demo_compiles()
    exe = os.path.join(ROOT, "demos", "random_tree")
    r = subprocess.run([exe, "naive", "5", "5", "0", "1"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "Kernel execution time:" in r.stdout and "Tree size: 71680" in r.stdout   # 10 x 7168 floats
    rows = (tmp_path / "samples.csv").read_text().splitlines()
    assert len(rows) == 10
    got = np.array([[float(v) for v in line.rstrip(",").split(",")] for line in rows])
    want = oracle_tree("naive", ROOT_STATE, 10, 32, 32).reshape(10, -1).astype(np.float64)
    assert np.all(np.abs(got - want) <= 5e-7 + 1e-6 * np.abs(want))   # "%f" printing
    r = subprocess.run([exe, "costprop"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Tree size: 3670016" in r.stdout
