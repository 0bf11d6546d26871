"""The drop-in boundary as a C++ caller sees it: include/planners/KGMT.h (the
reference class KGMT, include/planners/KGMT.cuh:23-109, over the C ABI) and
demos/main.cpp (the reference demos/main.cu with the CUDA calls swapped for the
ABI's helpers).  CPU: the demo compiles with plain g++ against libsbmp.so.  GPU:
it runs and prints / dumps what the reference's plan() does (KGMT.cu:100,294-311),
with the outcome of the oracle for the same seed."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, ROOT

DEMOS = os.path.join(ROOT, "demos")
LIB = os.path.join(ROOT, "cudasbmp_amd", "libsbmp.so")
CSVS = ("samples.csv", "unexploredSamples.csv", "parentRelations.csv", "uParentIdx.csv", "G.csv", "R2Avail.csv",
        "R1Avail.csv", "R1Valid.csv", "R2Valid.csv", "R1Invalid.csv", "R2Invalid.csv", "R1Score.csv", "R1.csv")


def _build():
    if not os.path.exists(LIB):
        pytest.skip("libsbmp.so not built")
    r = subprocess.run(["make", "-s", "-C", DEMOS], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(DEMOS, "main")


def test_demo_compiles_against_the_c_abi():
    exe = _build()
    assert os.access(exe, os.X_OK)
    nm = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True).stdout
    for sym in ("sbmp_kgmt_create", "sbmp_kgmt_plan", "sbmp_kgmt_export_csv", "sbmp_read_obstacles_csv",
                "sbmp_device_upload_f32", "sbmp_device_free"):
        assert sym in nm


@pytest.mark.gpu
def test_demo_runs_like_the_reference(tmp_path, oracle_lib, obstacles):
    exe = _build()
    run_dir = tmp_path / "build"
    run_dir.mkdir()
    cfg_dir = tmp_path / "configurations" / "obstacles"
    cfg_dir.mkdir(parents=True)
    (cfg_dir / "obstacles.csv").write_text(open(os.path.join(ROOT, "configurations", "obstacles",
                                                             "obstacles.csv")).read())
    seed = 12345
    r = subprocess.run([exe, "../configurations/obstacles/obstacles.csv", str(seed)], cwd=run_dir,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "numObstacles: 5" in out
    assert "Goal: 2.000000, 18.000000" in out
    assert "time inside KGMT is" in out
    m = re.findall(r"Iteration (\d+), Tree size (\d+)", out)
    assert m
    itr, tree = (int(x) for x in m[-1])
    o = oracle_lib.Oracle(oracle_lib.PlannerConfig(**DEMO), threads=4)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    info = o.info()
    assert (itr, tree) == (info["iterations"], info["treeSize"])
    for name in CSVS:
        assert (run_dir / name).exists(), name
    samples = np.loadtxt(run_dir / "samples.csv", delimiter=",", dtype=np.float64)
    assert samples.shape == (DEMO["maxTreeSize"], 7)
    s, p, c = o.tree()
    # std::fixed, 10 decimals (helper.cuh:53-72): each value is within 5e-11 of the float32 it printed.
    assert np.all(np.abs(samples[:tree] - s[:tree].astype(np.float64)) <= 6e-11)
    parents = np.loadtxt(run_dir / "parentRelations.csv", dtype=np.int64)
    assert np.array_equal(parents[:tree], p[:tree])
