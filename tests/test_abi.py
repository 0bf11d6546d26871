"""The C ABI library (libsbmp.so): loads, exports every symbol include/sbmp/sbmp.h
declares, and behaves without a GPU (no compute calls here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, OBSTACLES_CSV

HEADER = os.path.join(ROOT, "include", "sbmp", "sbmp.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sbmp_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def nat():
    from cudasbmp_amd import _native
    _native.lib()
    return _native


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ("sbmp_kgmt_create", "sbmp_kgmt_plan", "sbmp_kgmt_destroy", "sbmp_read_obstacles_csv",
              "sbmp_device_upload_f32", "sbmp_kgmt_create_sharded"):
        assert f in fns


def test_library_exports_every_declared_symbol(nat):
    L = nat.lib()
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, f"libsbmp.so lacks {missing}"
    assert set(header_functions()) == set(nat.EXPORTED_SYMBOLS)


def test_abi_version_and_status_strings(nat):
    L = nat.lib()
    assert L.sbmp_abi_version() == 1
    assert L.sbmp_status_string(0) == b"ok"
    assert L.sbmp_status_string(3) == b"I/O error"


def test_default_params_are_the_reference_demo(nat):
    p = nat.KgmtParams()
    nat.call("sbmp_kgmt_default_params", ctypes.byref(p))
    # reference demos/main.cu:19-28
    assert (p.width, p.height, p.N, p.n) == (20.0, 20.0, 16, 8)
    assert (p.numIterations, p.maxTreeSize, p.numDisc) == (100, 30000, 10)
    assert p.agentLength == 1.0 and abs(p.goalThreshold - 0.5) < 1e-7
    assert p.samplesPerIteration == 0 and p.batchRule == 0 and p.fixGNewClear == 0


def test_read_obstacles_csv_matches_reference_parser(tmp_path):
    from cudasbmp_amd import read_obstacles_csv
    obs = read_obstacles_csv(OBSTACLES_CSV)
    assert obs.shape == (5, 4)
    assert obs.tolist()[4] == [0, 6, 18, 8]
    # helper.cu:11-34: whitespace or single commas, count = floats / (2*dim), trailing floats dropped.
    f = tmp_path / "o.csv"
    f.write_text("1 2 3 4\n5,6,7,8\n\n9,10,11\n")
    o = read_obstacles_csv(str(f))
    assert o.shape == (2, 4) and o[1].tolist() == [5, 6, 7, 8]


def test_read_obstacles_missing_file_is_an_error_not_exit():
    from cudasbmp_amd import SbmpError, read_obstacles_csv
    with pytest.raises(SbmpError) as e:
        read_obstacles_csv("/nonexistent/obstacles.csv")
    assert e.value.status == 3


def test_invalid_params_are_rejected(nat):
    from cudasbmp_amd import KGMT, SbmpError
    with pytest.raises(SbmpError):
        KGMT(20.0, 20.0, 8, 8, 100, 30000, 10, 1.0, 0.5)   # N must be 16
    with pytest.raises(SbmpError):
        KGMT(20.0, 20.0, 16, 8, 100, 30000, 10, 1.0, 0.5, batchRule="fill")   # fill needs a cap


def test_no_device_fails_cleanly(nat):
    from cudasbmp_amd import KGMT, SbmpError, device_count
    if device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(SbmpError):
        KGMT(20.0, 20.0, 16, 8, 100, 30000, 10, 1.0, 0.5)


def test_missing_library_raises(monkeypatch):
    from cudasbmp_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libsbmp.so")
    with pytest.raises(_native.NativeLibraryError):
        _native.lib()


def test_system_config_loads():
    from cudasbmp_amd import load_system_config
    c = load_system_config()
    assert c["planner"]["maxTreeSize"] == 30000 and c["agent"] == "car"
    assert c["initial"][:2] == (5.0, 5.0) and c["goal"][:2] == (2.0, 18.0)
    assert os.path.exists(c["obstacles"])
    p = load_system_config(os.path.join(ROOT, "systems", "point.yaml"))
    assert p["agent"] == "point"


def test_reference_seed_conversion():
    from cudasbmp_amd import reference_seed_from_time
    # time(NULL) -> int -> unsigned long long (sign extension for negative ints)
    assert reference_seed_from_time(1723000000) == 1723000000
    assert reference_seed_from_time(2**31 + 5) == (2**64 - 2**31 + 5)


def test_kernel_objects_target_gfx950():
    from cudasbmp_amd import LIB_PATH
    data = open(LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert np.frombuffer(data[:4], dtype=np.uint8).tolist() == [0x7f, 0x45, 0x4c, 0x46]
