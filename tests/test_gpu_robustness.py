"""GPU: the error paths of plan() and the replica digest.

- A bounded in-kernel wait that gives up (status.error, kgmt_device.h kErr*) must end
  plan() with an error through the C ABI, whether or not the caller asks for a result
  (KgmtPlanner::run_to_goal, the single-rank plan loop; run(8), the others).  The wait is
  not made to time out (that would hold the GPU for a second per launch): begin() starts
  the plan with the error already set when SBMP_INJECT_WAIT_ERROR is given.
- sbmp_kgmt_state_hash: it changes when the state changes, it is reproducible, and a
  local shard group (whose ranks hold full replicas) digests to the single rank's value,
  since the two runs are bit-exact (tests/test_gpu_parity.py).
"""
import ctypes

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def d_obs(obstacles):
    from cudasbmp_amd import DeviceBuffer
    return DeviceBuffer(obstacles)


@pytest.mark.parametrize("code,word", [(1, "hand-off"), (2, "exchange")])
@pytest.mark.parametrize("local_group", [0, 2])
def test_plan_raises_wait_error(code, word, local_group, d_obs, obstacles, monkeypatch):
    from cudasbmp_amd import KGMT
    from cudasbmp_amd._native import SbmpError
    monkeypatch.setenv("SBMP_INJECT_WAIT_ERROR", str(code))
    g = KGMT(**DEMO, _local_group=local_group) if local_group else KGMT(**DEMO)
    with pytest.raises(SbmpError) as e:
        g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=1)
    assert word in str(e.value).lower() or "exchange" in str(e.value).lower()
    monkeypatch.delenv("SBMP_INJECT_WAIT_ERROR")
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=1)   # the next plan starts clean
    assert r.goalIndex >= 0


def test_plan_without_result_raises_wait_error(d_obs, obstacles, monkeypatch):
    """sbmp_kgmt_plan(..., result = NULL) still reports the error (it used to run
    result(), which reads the status, only when a result was asked for)."""
    from cudasbmp_amd import KGMT
    from cudasbmp_amd import _native as nat
    monkeypatch.setenv("SBMP_INJECT_WAIT_ERROR", "1")
    g = KGMT(**DEMO)
    i = np.array(DEMO_INITIAL, dtype=np.float32)
    gl = np.array(DEMO_GOAL, dtype=np.float32)
    with pytest.raises(nat.SbmpError):
        nat.call("sbmp_kgmt_plan", g._h, i.ctypes.data_as(ctypes.c_void_p), gl.ctypes.data_as(ctypes.c_void_p),
                 ctypes.c_void_p(d_obs.ptr), len(obstacles), 1, None)


def test_plan_stops_early_on_wait_error(d_obs, obstacles, monkeypatch):
    """The single-rank plan loop stops enqueueing once a planner reports the error: far
    fewer than numIterations launches run."""
    from cudasbmp_amd import KGMT
    from cudasbmp_amd._native import SbmpError
    monkeypatch.setenv("SBMP_INJECT_WAIT_ERROR", "1")
    cfg = dict(DEMO, numIterations=2000, maxTreeSize=1 << 20, goalThreshold=0.0)
    g = KGMT(**cfg)
    with pytest.raises(SbmpError):
        g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=1)
    ran = len(g.iter_log())   # the injected error does not stop the kernels, only the host loop
    assert 0 < ran <= 8, ran


def _digest(g, d_obs, obstacles, seed, iters=None):
    if iters is None:
        g.plan(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed=seed)
    else:
        g.begin(DEMO_INITIAL, DEMO_GOAL, d_obs, len(obstacles), seed)
        g.enqueue(iters)
        g.sync()
    return g.state_hash()


def test_state_hash_tracks_the_state(d_obs, obstacles):
    from cudasbmp_amd import KGMT
    cfg = dict(DEMO, goalThreshold=0.0, samplesPerIteration=4096, maxTreeSize=200000, numIterations=30)
    g = KGMT(**cfg, batchRule="fill")
    h5 = _digest(g, d_obs, obstacles, 3, iters=5)
    assert _digest(g, d_obs, obstacles, 3, iters=5) == h5, "digest is not reproducible"
    assert _digest(g, d_obs, obstacles, 3, iters=6) != h5, "one more iteration left the digest unchanged"
    assert _digest(g, d_obs, obstacles, 4, iters=5) != h5, "another seed left the digest unchanged"
    assert h5 != 0


@pytest.mark.parametrize("P", [2, 3])
def test_local_group_digest_equals_single_rank(P, d_obs, obstacles):
    """LocalShardGroup::state_hash (every rank's digest, checked equal inside) against the
    single-rank planner on the same seed: the replicated state is the same bits."""
    from cudasbmp_amd import KGMT
    cfg = dict(DEMO, goalThreshold=0.0, samplesPerIteration=4096, maxTreeSize=200000, numIterations=12)
    single = _digest(KGMT(**cfg, batchRule="fill"), d_obs, obstacles, 9)
    group = _digest(KGMT(**cfg, batchRule="fill", _local_group=P), d_obs, obstacles, 9)
    assert group == single
