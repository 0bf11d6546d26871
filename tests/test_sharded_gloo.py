"""Multi-process sharded planning over torch.distributed (gloo, world_size 2, CPU).

Each process owns the slots of one rank (block-cyclic 256-slot blocks, SURVEY.md
§8e) and runs the oracle's local expansion; per iteration the ranks exchange
their accepted-child records (all_gather of count + padded payload) and sum
their region deltas (all_reduce), then every rank inserts the slot-sorted union.
This is the data flow of the GPU sharded planner (RCCL allgather / allreduce
over xGMI); the test proves it reproduces the single-rank planner bit for bit.
"""
import os
import socket

import numpy as np
import pytest

from conftest import DEMO, DEMO_GOAL, DEMO_INITIAL, OBSTACLES_CSV, ROOT

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange(dist, torch, recs, deltas):
    """all_gather variable-length record arrays; all_reduce the delta vector."""
    raw = np.frombuffer(recs.tobytes(), dtype=np.uint8)
    n = torch.tensor([len(raw)], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    cap = int(max(s.item() for s in sizes))
    buf = torch.zeros(max(cap, 1), dtype=torch.uint8)
    buf[:len(raw)] = torch.from_numpy(raw.copy())
    out = [torch.zeros(max(cap, 1), dtype=torch.uint8) for _ in range(dist.get_world_size())]
    dist.all_gather(out, buf)
    parts = [o[:int(s.item())].numpy().tobytes() for o, s in zip(out, sizes)]
    d = torch.from_numpy(deltas.astype(np.int64))
    dist.all_reduce(d)
    return parts, d.numpy().astype(np.int32)


def _worker(rank, port, cfg_kw, seed, result_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    obstacles = np.loadtxt(OBSTACLES_CSV, delimiter=",", dtype=np.float32).reshape(-1, 4)
    cfg = pyoracle.PlannerConfig(**{**DEMO, **cfg_kw})
    o = pyoracle.Oracle(cfg, threads=2, nranks=WORLD, rank=rank)
    o.begin(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    while True:
        ret = o.expand_local()
        flag = torch.tensor([1 if ret >= 0 else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item() == 0:
            break
        parts, deltas = _exchange(dist, torch, o.local_records(), o.local_deltas())
        recs = np.concatenate([np.frombuffer(p, dtype=pyoracle.RECORD_DTYPE) for p in parts])
        o.finish(recs, deltas)
        if o.info()["terminated"]:
            break
    s, p, c = o.tree()
    n = o.info()["treeSize"]
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), s=s[:n], p=p[:n], c=c[:n],
             log=o.iter_logs(), goal=np.int64(o.info()["goalIdx"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_kw,seed", [
    (dict(), 3),
    (dict(samplesPerIteration=4096, batchRule=1, maxTreeSize=120000, numIterations=8, goalThreshold=0.0), 8),
])
def test_gloo_two_ranks_match_single_rank(tmp_path, oracle_lib, obstacles, cfg_kw, seed):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_worker, args=(port, cfg_kw, seed, str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    ref = oracle_lib.Oracle(oracle_lib.PlannerConfig(**{**DEMO, **cfg_kw}), threads=4)
    ref.plan(DEMO_INITIAL, DEMO_GOAL, obstacles, seed)
    n = ref.info()["treeSize"]
    rs, rp, rc = ref.tree()
    for r in range(WORLD):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert int(z["goal"]) == ref.info()["goalIdx"]
        assert z["log"].tolist() == ref.iter_logs().tolist()
        assert np.array_equal(z["s"].view(np.uint32), rs[:n].view(np.uint32))
        assert np.array_equal(z["p"], rp[:n])
        assert np.array_equal(z["c"].view(np.uint32), rc[:n].view(np.uint32))
