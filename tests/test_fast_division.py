"""Host check of k_expand / k_step's slot -> frontier-position division (div_small,
cudasbmp_amd/csrc/kgmt_kernels.hip): q0 = trunc(f32(a) * rcp(b)), then at most two
integer correction steps each way.  v_rcp_f32 is within 1 ulp of 1/b, so the check
runs with RN(1/b) and its two neighbours.  It must give a // b for every a below
kFastDivMax = 2^24 (larger slot counts take the exact integer division), and the
two-step correction must be enough; the ADVICE round-1 counterexample (a = 67,108,867,
b = 1) sits above the bound and shows why the bound is needed.
"""
import numpy as np

FAST_DIV_MAX = 1 << 24


def div_small(a: np.ndarray, b: int, rcp: np.float32) -> np.ndarray:
    q = np.trunc(a.astype(np.float32) * rcp).astype(np.int64)   # f32 product, one rounding
    r = a - q * b
    for _ in range(2):
        m = r < 0
        q[m] -= 1
        r[m] += b
    for _ in range(2):
        m = r >= b
        q[m] += 1
        r[m] -= b
    return q


def _inputs(b: int, rng) -> np.ndarray:
    top = np.arange(FAST_DIV_MAX - (1 << 15), FAST_DIV_MAX, dtype=np.int64)
    rnd = rng.integers(0, FAST_DIV_MAX, size=1 << 15, dtype=np.int64)
    q = rng.integers(0, FAST_DIV_MAX // b, size=1 << 13, dtype=np.int64)
    edges = np.concatenate([q * b - 1, q * b, q * b + b - 1])
    a = np.concatenate([top, rnd, edges, np.arange(0, 4096, dtype=np.int64)])
    return a[(a >= 0) & (a < FAST_DIV_MAX)]


def test_div_small_exact_below_bound():
    rng = np.random.default_rng(1)
    for b in list(range(1, 65)) + [100, 255, 256, 257, 1000, 4095, 65535, 1 << 20]:
        r0 = np.float32(1.0) / np.float32(b)
        for rcp in (np.nextafter(r0, np.float32(0)), r0, np.nextafter(r0, np.float32(1))):
            a = _inputs(b, rng)
            got = div_small(a, b, np.float32(rcp))
            assert np.array_equal(got, a // b), f"b={b} rcp={rcp!r}"


def test_div_small_needs_the_bound():
    a = np.array([67_108_867], dtype=np.int64)   # wrong quotient for k = 1 above 2^24
    assert div_small(a, 1, np.float32(1.0))[0] != a[0]
