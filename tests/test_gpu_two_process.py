"""The cross-process sharded HIP path with two real processes on one GPU.

Each process is one rank of sbmp_kgmt_create_sharded_host: the real sharded k_step
kernel (one launch per iteration), each rank's lists of accepted children written to
its record buffer with system-scope stores and read by the peer over HIP IPC
(hipIpcGetMemHandle / hipIpcOpenMemHandle, handles exchanged by an allgather), and
the fused exchange buffer all-reduced every iteration, either by the default one-shot exchange (each rank stores its buffer into
every rank's IPC-mapped inbox and raises flags; both processes' kernels meet on the
GPU; the inboxes are uncached device memory) as its own k_oneshot launch, or, with
SBMP_EXCHANGE=collective, by the Exchange's all-reduce.  With the one-shot exchange the
same kernel also pushes each rank's lists into every rank's list mirror, and k_step reads
its parents from its own memory (SBMP_MIRROR=0: from the peer's record buffer); by
default the exchange itself then runs in k_step's tail, done by the last arrivals of its
expanding workgroups, with no k_oneshot launch (SBMP_FUSED_EXCHANGE=0: the separate kernel).
RCCL cannot put two ranks on one device, so that all-reduce and the IPC handle
exchange run over torch.distributed gloo through the host-collectives seam
(cudasbmp_amd/host_comm.py).  The ranks' merged state must equal the CPU oracle's
single-rank run bit for bit.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, ROOT, bits
from test_gpu_parity import _oracle

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, port, kw, seed, out_dir, exchange, delay=0.0):
    import sys
    import time
    sys.path.insert(0, ROOT)
    if exchange == "collective":
        os.environ["SBMP_EXCHANGE"] = exchange
    else:
        os.environ.pop("SBMP_EXCHANGE", None)
    if exchange == "oneshot-remote":   # k_step reads the peers' record buffers over the mapping
        os.environ["SBMP_MIRROR"] = "0"
    else:
        os.environ.pop("SBMP_MIRROR", None)
    if exchange == "oneshot-kernel":   # the exchange as its own k_oneshot launch, not in k_step's tail
        os.environ["SBMP_FUSED_EXCHANGE"] = "0"
    else:
        os.environ.pop("SBMP_FUSED_EXCHANGE", None)
    if exchange == "oneshot-check-fails" and rank == 1:   # only rank 1's start-up check "fails"
        os.environ["SBMP_ONESHOT_SELFTEST"] = "fail"
    else:
        os.environ.pop("SBMP_ONESHOT_SELFTEST", None)
    if exchange == "mirror-check-fails" and rank == 1:   # only rank 1's list-mirror check "fails"
        os.environ["SBMP_MIRROR_SELFTEST"] = "fail"
    else:
        os.environ.pop("SBMP_MIRROR_SELFTEST", None)
    if exchange == "fused-check-fails" and rank == 1:   # only rank 1's fused-exchange check "fails"
        os.environ["SBMP_FUSED_SELFTEST"] = "fail"
    else:
        os.environ.pop("SBMP_FUSED_SELFTEST", None)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from cudasbmp_amd import DeviceBuffer, KGMT
    from cudasbmp_amd.host_comm import TorchCollectives
    obs = np.loadtxt(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"), delimiter=",",
                     dtype=np.float32).reshape(-1, 4)
    cfg = dict(DEMO)
    extra = {k: kw[k] for k in ("samplesPerIteration", "batchRule", "fixGNewClear") if k in kw}
    cfg.update({k: v for k, v in kw.items() if k not in extra})
    g = KGMT(**cfg, **extra, _host_sharded=(TorchCollectives(dist), WORLD, rank))
    if rank == 1 and delay:
        time.sleep(delay)   # process skew before the first exchange (begin() holds a host barrier)
    g.set_profiling(True)   # counts the launches: which exchange ran
    r = g.plan(DEMO_INITIAL, DEMO_GOAL, DeviceBuffer(obs), len(obs), seed=seed)
    oneshots = g.kernel_stats().get("k_oneshot", (0, 0.0))[0]
    pinfo = g.path_info()
    mirror, fused = pinfo["list_mirror"], pinfo["fused_exchange"]
    checks = np.array([pinfo["oneshot_check"], pinfo["mirror_check"], pinfo["fused_check"]])
    digest = np.uint64(g.state_hash())   # the replicated state: the same on both ranks
    s, p, c = g.tree()
    G, GN = g.flags()          # GNew words live with their owner: merged by the all-reduce
    reg = g.regions()          # R2Valid / R2Invalid: each rank folded its own children
    u, up = g.unexplored()     # slots of other ranks read as 0 / -1
    rng = g.rng()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), s=s, p=p, c=c, G=G, GN=GN, u=u, up=up, rng=rng,
             log=g.iter_log(), res=np.array([r.iterations, r.treeSize, r.goalIndex]), oneshots=oneshots, mirror=mirror, fused=fused,
             checks=checks, digest=digest,
             cost=np.float32(r.costToGoal), **{"reg_" + k: v for k, v in reg.items()})
    g.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("kw,seed,exchange,delay", [
    (dict(), 3, "oneshot", 0.0),
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "oneshot", 0.0),
    (dict(fixGNewClear=True, numIterations=40), 8, "oneshot", 0.0),
    (dict(), 3, "collective", 0.0),
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "collective", 0.0),
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "oneshot-remote", 0.0),
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "oneshot-kernel", 0.0),
    (dict(fixGNewClear=True, numIterations=40), 8, "oneshot-kernel", 0.0),
    # rank 1 starts 3 s late (round 2's exchange gave up after 1 s)
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "oneshot", 3.0),
    # rank 1's start-up check of the one-shot exchange fails: both ranks must switch to the
    # all-reduce together (one rank alone would leave the other waiting for its flags)
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "oneshot-check-fails", 0.0),
    # rank 1's start-up check of the list mirror fails: both ranks must drop the mirror (and with
    # it the fused exchange) together and read the lists over the mapping with k_oneshot
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "mirror-check-fails", 0.0),
    # rank 1's start-up check of the fused exchange's in-kernel order fails: both ranks keep
    # the mirror and run the exchange as its own k_oneshot launch, together
    (dict(samplesPerIteration=4096, batchRule="fill", maxTreeSize=200000, numIterations=15, goalThreshold=0.0), 21,
     "fused-check-fails", 0.0),
])
def test_two_processes_one_gpu_bit_exact(kw, seed, exchange, delay, tmp_path, obstacles, oracle_lib):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, port, kw, seed, str(tmp_path), exchange, delay))
             for r in range(WORLD)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    for pr in procs:
        if pr.is_alive():
            pr.kill()
            pr.join()
    assert [pr.exitcode for pr in procs] == [0] * WORLD, f"rank exit codes {[pr.exitcode for pr in procs]}"
    R = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(WORLD)]

    cfg = dict(DEMO)
    extra = {k: kw[k] for k in ("samplesPerIteration", "batchRule", "fixGNewClear") if k in kw}
    cfg.update({k: v for k, v in kw.items() if k not in extra})
    o = _oracle(cfg, extra)
    o.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    so, po, co = o.tree()
    Go, GNo = o.flags()
    uo, upo = o.unexplored()
    ro = o.regions()
    info = o.info()
    n = o.rng().shape[0]
    owner = (np.arange(n) // 256) % WORLD
    for r, d in enumerate(R):
        # default: the lists go into every rank's mirror and the exchange runs in k_step's tail
        # (no k_oneshot launch); SBMP_FUSED_EXCHANGE=0 launches k_oneshot; SBMP_MIRROR=0 reads the
        # lists over the mapping, with k_oneshot; the collective exchange uses neither
        fused = exchange == "oneshot"
        assert bool(d["fused"]) == fused, f"rank {r}: fused exchange {bool(d['fused'])}"
        assert bool(d["mirror"]) == (exchange in ("oneshot", "oneshot-kernel", "fused-check-fails")), \
            f"rank {r}: list mirror {bool(d['mirror'])}"
        if exchange in ("oneshot-kernel", "oneshot-remote", "mirror-check-fails", "fused-check-fails"):
            assert int(d["oneshots"]) > 0, f"rank {r}: the one-shot exchange did not run"
        else:
            assert int(d["oneshots"]) == 0, f"rank {r}: k_oneshot ran ({int(d['oneshots'])} launches)"
        # the start-up checks: which ran, and the all-reduced verdict every rank acted on
        want = {"collective": ["not run"] * 3, "oneshot-check-fails": ["failed", "not run", "not run"],
                "oneshot-remote": ["passed", "not run", "not run"],
                "mirror-check-fails": ["passed", "failed", "not run"],
                "oneshot-kernel": ["passed", "passed", "not run"],
                "fused-check-fails": ["passed", "passed", "failed"]}.get(exchange, ["passed"] * 3)
        assert d["checks"].tolist() == want, f"rank {r}: start-up checks {d['checks'].tolist()}"
    assert len({int(d["digest"]) for d in R}) == 1, "the ranks' replicated states differ"
    for r, d in enumerate(R):   # every rank holds the whole tree and the merged exports
        assert np.array_equal(d["log"], o.iter_logs()), f"rank {r}: iteration logs differ"
        assert np.array_equal(d["p"], po), f"rank {r}: parents differ"
        assert np.array_equal(bits(d["s"]), bits(so)), f"rank {r}: tree samples differ"
        assert np.array_equal(bits(d["c"]), bits(co)), f"rank {r}: costs differ"
        assert np.array_equal(d["G"], Go) and np.array_equal(d["GN"], GNo), f"rank {r}: G / GNew differ"
        for k in ro:
            assert np.array_equal(bits(d["reg_" + k]), bits(ro[k])), f"rank {r}: {k} differs"
        assert d["res"].tolist() == [info["iterations"], info["treeSize"], info["goalIdx"]]
        assert bits(np.float32(d["cost"])) == bits(np.float32(info["costToGoal"]))
        own = owner == r   # slot state lives with its owner only
        assert np.array_equal(d["rng"][own], o.rng()[own]), f"rank {r}: RNG states differ"
        assert np.array_equal(d["up"][:n][own], upo[:n][own]) and \
            np.array_equal(bits(d["u"][:n][own]), bits(uo[:n][own])), f"rank {r}: unexplored slots differ"
        assert (d["up"][:n][~own] == -1).all()
