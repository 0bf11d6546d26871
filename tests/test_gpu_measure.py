"""The bench's measured HBM copy rate (sbmp_hbm_copy_bandwidth): a sane
figure below the 8 TB/s spec, and argument checks through the C ABI."""
import pytest

pytestmark = pytest.mark.gpu


def test_copy_bandwidth_is_below_spec():
    from cudasbmp_amd.kgmt import hbm_copy_bandwidth
    gbs = hbm_copy_bandwidth(1 << 30, 3)
    assert 1000.0 < gbs < 8000.0, gbs


def test_copy_bandwidth_rejects_tiny_buffers():
    from cudasbmp_amd import SbmpError
    from cudasbmp_amd.kgmt import hbm_copy_bandwidth
    with pytest.raises(SbmpError):
        hbm_copy_bandwidth(1024, 3)
