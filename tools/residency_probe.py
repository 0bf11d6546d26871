"""k_step residency as begin() sees it (path_info) at the c3 shape, per planner form:
single rank, a local shard group of 2, and one host-sharded rank (gloo, world 1).

    python tools/residency_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv  # noqa: E402


def probe(name, **extra):
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    d_obs = DeviceBuffer(obs)
    P = extra.pop("P", 1)
    k = KGMT(20.0, 20.0, 16, 8, 60, 1 << 24, 10, 1.0, 0.0, samplesPerIteration=262144 * P, batchRule="fill",
             fixGNewClear=True, **extra)
    try:
        k.begin((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), d_obs, len(obs), 20240807)
        print(name, k.path_info(), flush=True)
    except Exception as e:   # noqa: BLE001 - the message is the probe's result
        print(name, "begin failed:", e, flush=True)
    k.close()


def main():
    probe("single")
    probe("local2", P=2, _local_group=2)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import torch.distributed as dist
    from cudasbmp_amd.host_comm import TorchCollectives
    dist.init_process_group("gloo", rank=0, world_size=1)
    probe("host1", _host_sharded=(TorchCollectives(dist), 1, 0))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
