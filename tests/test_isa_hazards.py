"""The VMEM store-data hazard in the built gfx950 code (CPU only: disassembly, no GPU).

ROCm 7.2 leaves a >8-B MUBUF store whose soffset is an SGPR unpadded, and a VALU write of
its data VGPRs in the next instruction then changes what the store writes (round 3:
`test_c2_point_bit_exact` lost vx in thousands of rows).  The kernels keep
soffset 0; tools/isa_hazards.py checks the library, not the convention.
"""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_hazards  # noqa: E402

LIB = os.path.join(ROOT, "cudasbmp_amd", "libsbmp.so")
HIPCC = "/opt/rocm/bin/hipcc"


def test_scanner_on_synthetic_isa():
    bad = ["\tbuffer_store_dwordx4 v[8:11], v1, s[8:11], s12 offen offset:16 // 0000: E07C",
           "\tv_mov_b32_e32 v8, v7 // 0008: 7E10"]
    assert len(isa_hazards.scan_lines(bad)) == 1
    padded = [bad[0], "\ts_nop 0", bad[1]]
    assert isa_hazards.scan_lines(padded) == []
    other_reg = [bad[0], "\tv_mov_b32_e32 v12, v7"]
    assert isa_hazards.scan_lines(other_reg) == []
    narrow = ["\tbuffer_store_dwordx2 v[8:9], v1, s[8:11], s12 offen", "\tv_mov_b32_e32 v8, v7"]
    assert isa_hazards.scan_lines(narrow) == []
    glob = ["\tglobal_store_dwordx4 v[2:3], v[4:7], off", "\tv_add_f32_e32 v6, v1, v2"]
    assert len(isa_hazards.scan_lines(glob)) == 1
    scalar_dst = [bad[0], "\tv_readfirstlane_b32 s8, v8"]
    assert isa_hazards.scan_lines(scalar_dst) == []


def test_library_has_no_store_data_hazard():
    if not os.path.exists(LIB):
        pytest.skip("libsbmp.so not built (python -m cudasbmp_amd.build)")
    n, stores, hazards = isa_hazards.scan_library(LIB)
    assert n >= 1 and stores > 100
    assert hazards == [], f"{len(hazards)} unpadded wide stores: {hazards[:4]}"


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="hipcc not available")
def test_scanner_catches_the_round3_store_form(tmp_path):
    """The list stores of k_step with the block part in an SGPR soffset (-DSBMP_SOFFSET_DEMO)
    reproduce round 3's unpadded store; the scan must report it."""
    src = os.path.join(ROOT, "cudasbmp_amd", "csrc", "kgmt_kernels.hip")
    from cudasbmp_amd.build import COMMON
    obj = str(tmp_path / "k.o")
    so = str(tmp_path / "libdemo.so")
    subprocess.run([HIPCC] + COMMON + ["-DSBMP_SOFFSET_DEMO", "-x", "hip", "-c", src, "-o", obj], check=True,
                   capture_output=True)
    subprocess.run([HIPCC, "-shared", "--offload-arch=gfx950", obj, "-o", so], check=True, capture_output=True)
    _, _, hazards = isa_hazards.scan_library(so)
    assert hazards, "the SGPR-soffset list stores compiled without a hazard: the demo no longer reproduces it"
    assert all("buffer_store_dwordx4" in s for s, _ in hazards)


def test_hot_kernels_use_no_scratch():
    """Every k_step and k_expand instantiation keeps its state in registers: no scratch
    (private segment) and no VGPR spills.  Round 6: indexing the register obstacle list by
    lane put it in scratch and made k_expand 25% slower."""
    if not os.path.exists(LIB):
        pytest.skip("libsbmp.so not built (python -m cudasbmp_amd.build)")
    res = isa_hazards.kernel_resources(LIB)
    hot = {k: v for k, v in res.items() if "k_step" in k or "k_expand" in k}
    assert len(hot) >= 40, sorted(res)[:8]
    bad = {k: v for k, v in hot.items() if v[1] or v[2]}
    assert not bad, f"{len(bad)} hot kernels spill or use scratch: {list(bad.items())[:4]}"
