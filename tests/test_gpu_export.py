"""The reference's on-disk formats, written by demos/main (the
reference demo over the C ABI) and compared TEXT-for-text with what the CPU oracle's
state prints in the same format (helper.cuh:53-79: std::fixed, 10 decimals, one row
per element, comma-separated columns):
  - the 13 final CSVs of KGMT.cu:299-311, all of them;
  - the per-iteration Data/<Kind>/<kind><itr>.csv dumps of KGMT.cu:263-290
    (--dump-iterations), against the oracle stepped one iteration at a time;
  - --config systems/car.yaml (the library's config parser) gives the same run as the
    hardcoded demo constants of main.cu:19-46.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, ROOT
from test_demo import CSVS, _build

pytestmark = pytest.mark.gpu


def csv_text(a) -> str:
    """helper.cuh:53-72 writeVectorToCSV: floats as std::fixed << setprecision(10), ints as ints."""
    a = np.asarray(a)
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    if a.dtype.kind == "f":
        rows = (",".join(f"{float(v):.10f}" for v in r) for r in a)
    else:
        rows = (",".join(str(int(v)) for v in r) for r in a)
    return "".join(r + "\n" for r in rows)


def _run_demo(tmp_path, extra, seed):
    exe = _build()
    run_dir = tmp_path / "build"
    run_dir.mkdir()
    r = subprocess.run([exe] + extra + [str(seed)], cwd=run_dir, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return run_dir, r.stdout


def _oracle_files(o):
    s, p, c = o.tree()
    u, up = o.unexplored()
    G, _ = o.flags()
    reg = o.regions()
    return {"samples.csv": s, "unexploredSamples.csv": u, "parentRelations.csv": p, "uParentIdx.csv": up,
            "G.csv": G.astype(np.int32), "R2Avail.csv": reg["R2Avail"], "R1Avail.csv": reg["R1Avail"],
            "R1Valid.csv": reg["R1Valid"], "R2Valid.csv": reg["R2Valid"], "R1Invalid.csv": reg["R1Invalid"],
            "R2Invalid.csv": reg["R2Invalid"], "R1Score.csv": reg["R1Score"], "R1.csv": reg["R1"]}


def test_all_final_csvs_and_per_iteration_dumps(tmp_path, oracle_lib, obstacles):
    seed = 4242
    cfg = os.path.join(ROOT, "systems", "car.yaml")
    run_dir, out = _run_demo(tmp_path, ["--config", cfg, "--dump-iterations", "."], seed)
    itr, tree = (int(x) for x in re.findall(r"Iteration (\d+), Tree size (\d+)", out)[-1])
    o = oracle_lib.Oracle(oracle_lib.PlannerConfig(**DEMO), threads=8)
    o.begin(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    kinds = [("Samples", "samples"), ("Parents", "parents"), ("R1Scores", "R1Scores"), ("R1Avail", "R1Avail"),
             ("R1", "R1"), ("UnexploredSamples", "unexploredSamples")]
    t = 0
    while o.step():
        t += 1
        s, p, c = o.tree()
        u, _ = o.unexplored()
        reg = o.regions()
        want = {"Samples": s, "Parents": p, "R1Scores": reg["R1Score"], "R1Avail": reg["R1Avail"], "R1": reg["R1"],
                "UnexploredSamples": u}
        for d, stem in kinds:
            got = (run_dir / "Data" / d / f"{stem}{t}.csv").read_text()
            assert got == csv_text(want[d]), f"Data/{d}/{stem}{t}.csv differs"
    assert t == itr >= 2 and o.info()["treeSize"] == tree
    assert not (run_dir / "Data" / "Samples" / f"samples{t + 1}.csv").exists()
    assert (run_dir / "Data" / "G").is_dir() and (run_dir / "Data" / "GNew").is_dir()   # created, left empty
    want = _oracle_files(o)
    for name in CSVS:
        assert (run_dir / name).read_text() == csv_text(want[name]), f"{name} differs"


def test_config_file_equals_hardcoded_demo(tmp_path):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    obs = os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv")
    a_dir, a_out = _run_demo(tmp_path / "a", [obs], 77)
    b_dir, b_out = _run_demo(tmp_path / "b", ["--config", os.path.join(ROOT, "systems", "car.yaml")], 77)
    strip = lambda s: re.sub(r"time inside KGMT is \S+", "", s)   # noqa: E731
    assert strip(a_out) == strip(b_out)
    for name in CSVS:
        assert (a_dir / name).read_bytes() == (b_dir / name).read_bytes(), name
