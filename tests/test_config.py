"""System files: the library's parser (sbmp_load_system_config,
cudasbmp_amd/csrc/config.cpp) on every file under systems/, its error behaviour, and
the reference's configurations/ files (init, goal, numR1, R2) it can read.  No GPU."""
import os

import pytest

from conftest import ROOT

SYSTEMS = os.path.join(ROOT, "systems")


def test_demo_file_is_main_cu():
    from cudasbmp_amd.config import load_system_config
    c = load_system_config(os.path.join(SYSTEMS, "car.yaml"))
    assert c["planner"] == dict(width=20.0, height=20.0, N=16, n=8, numIterations=100, maxTreeSize=30000, numDisc=10,
                                agentLength=1.0, goalThreshold=0.5)   # demos/main.cu:19-28
    assert c["agent"] == "car" and c["initial"][:2] == (5.0, 5.0) and c["goal"][:2] == (2.0, 18.0)
    assert os.path.samefile(c["obstacles"], os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))


@pytest.mark.parametrize("name,agent,S,boxes", [("c1", "point", 1024, "obstacles.csv"),
                                                ("c2", "point", 262144, "obstacles.csv"),
                                                ("c3", "car", 262144, "obstacles.csv"),
                                                ("c4", "car", 131072, "obstacles.csv"),
                                                ("c5", "car", 131072, "obstacles_c5.csv")])
def test_workload_files(name, agent, S, boxes):
    from cudasbmp_amd.config import workload
    c = workload(name)
    assert c["agent"] == agent and c["samplesPerIteration"] == S and c["batchRule"] == "fill"
    assert c["fixGNewClear"] and c["planner"]["goalThreshold"] == 0.0
    assert os.path.basename(c["obstacles"]) == boxes and os.path.exists(c["obstacles"])


def test_reference_configuration_files():
    """configurations/{init,goal,numR1,R2}: start (1, 1), goal (9, 9), N = n = 16."""
    from cudasbmp_amd.config import load_system_config
    c = load_system_config(os.path.join(SYSTEMS, "car_reference_files.yaml"))
    assert c["initial"] == (1.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0) and c["goal"][:2] == (9.0, 9.0)
    assert c["planner"]["N"] == 16 and c["planner"]["n"] == 16
    assert c["planner"]["maxTreeSize"] == 30000   # not in the file: the demo default


@pytest.mark.parametrize("text,msg", [("widht: 20\n", "unknown key"), ("N: 1.5\n", "integer"),
                                      ("agent: boat\n", "car or point"), ("batchRule: all\n", "reference or fill"),
                                      ("initial: [1]\n", "2 to 7"), ("width 20\n", "key: value"),
                                      ("goal: nowhere.csv\n", "neither numbers nor a readable file")])
def test_errors(tmp_path, text, msg):
    from cudasbmp_amd import SbmpError
    from cudasbmp_amd.config import load_system_config
    p = tmp_path / "bad.yaml"
    p.write_text(text)
    with pytest.raises(SbmpError, match=msg):
        load_system_config(str(p))


def test_missing_file_is_an_io_error(tmp_path):
    from cudasbmp_amd import SbmpError
    from cudasbmp_amd.config import load_system_config
    with pytest.raises(SbmpError, match="cannot open"):
        load_system_config(str(tmp_path / "none.yaml"))


def test_comments_quotes_and_relative_paths(tmp_path):
    from cudasbmp_amd.config import load_system_config
    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / "start.csv").write_text("3.5, 4.5\n")
    p = tmp_path / "x.yaml"
    p.write_text("# a comment\n\nagent: point   # trailing\nobstacles: 'boxes.csv'\ninitial: sub/start.csv\n"
                 "fixGNewClear: true\nsamplesPerIteration: 4096\nbatchRule: fill\n")
    c = load_system_config(str(p))
    assert c["agent"] == "point" and c["initial"] == (3.5, 4.5, 0.0, 0.0, 0.0, 0.0, 0.0)
    assert c["obstacles"] == str(tmp_path / "boxes.csv") and c["samplesPerIteration"] == 4096
