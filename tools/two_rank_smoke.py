"""Two sharded ranks (separate processes, GPUs 0 and 1) over RCCL + IPC, compared
with the oracle: the multi-process path end to end.  Needs two GPUs (RCCL rejects
two ranks on one device with "invalid usage").  python tools/two_rank_smoke.py"""
import ctypes
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv
    from cudasbmp_amd import _native as nat
    uid = (ctypes.c_uint8 * nat.SBMP_COMM_ID_BYTES)()
    if rank == 0:
        nat.call("sbmp_comm_get_unique_id", uid)
    obj = [bytes(uid)]
    dist.broadcast_object_list(obj, src=0)
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    k = KGMT(20.0, 20.0, 16, 8, 20, 200000, 10, 1.0, 0.0, samplesPerIteration=4096, batchRule="fill",
             device=rank, _sharded=(obj[0], 2, rank))
    k.plan((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), DeviceBuffer(obs), len(obs), seed=21)
    s, p, c = k.tree()
    q.put((rank, k.treeSize_, s[:k.treeSize_].tobytes(), p[:k.treeSize_].tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    from oracle.pyoracle import Oracle, PlannerConfig
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for pr in procs:
        pr.join(timeout=60)
    obs = np.loadtxt(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"), delimiter=",",
                     dtype=np.float32).reshape(-1, 4)
    o = Oracle(PlannerConfig(numIterations=20, maxTreeSize=200000, goalThreshold=0.0, samplesPerIteration=4096,
                             batchRule=1), threads=8)
    o.plan((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), obs, 21)
    s, p, c = o.tree()
    n = o.info()["treeSize"]
    for rank, ts, sb, pb in sorted(res):
        ok = ts == n and sb == s[:n].tobytes() and pb == p[:n].tobytes()
        print(f"rank {rank}: treeSize {ts} (oracle {n}) bit-exact {ok}")
        assert ok
    print("TWO-RANK OK")


if __name__ == "__main__":
    main()
