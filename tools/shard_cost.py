"""Per-rank kernel costs of the sharded data flow at bench scale, on one GPU: a
local shard group of P virtual ranks with P x 262,144 children per iteration (the
weak-scaling bench at N = P), so every rank's k_step sees P x 1024 global
blocks.  The ranks run one after another on one stream, so only the per-kernel
means are meaningful, not the wall time.  P = h1: one host-sharded rank (world 1).
python tools/shard_cost.py [P ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv  # noqa: E402


def host_rank():
    """One host-sharded rank (gloo, world 1): the sharded k_step + k_oneshot (+ list mirror)
    sequence a rank of a multi-GPU run executes, without peers."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    import torch.distributed as dist
    from cudasbmp_amd.host_comm import TorchCollectives
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    return (TorchCollectives(dist), 1, 0)


def main():
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    d_obs = DeviceBuffer(obs)
    for a in sys.argv[1:] or ["1", "2", "4", "8"]:
        P = 1 if a == "h1" else int(a)
        extra = {"_host_sharded": host_rank()} if a == "h1" else {"_local_group": P if P > 1 else 0}
        k = KGMT(20.0, 20.0, 16, 8, 90, 1 << 24, 10, 1.0, 0.0, samplesPerIteration=262144 * P, batchRule="fill",
                 fixGNewClear=True, **extra)
        k.begin((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), d_obs, len(obs), 20240807)
        k.enqueue(20)
        k.sync()
        k.set_profiling(True)
        k.reset_kernel_stats()
        k.enqueue(30)
        k.sync()
        st = k.kernel_stats()
        k.set_profiling(False)
        t0 = time.perf_counter()   # unprofiled: the iteration's wall time (a local group's ranks take turns)
        k.enqueue(30)
        k.sync()
        wall = (time.perf_counter() - t0) / 30 * 1e6
        print(f"P={a} (rank 0): " + ", ".join(f"{n} {1e3 * ms / max(1, c):.2f} us x{c}" for n, (c, ms) in st.items())
              + f"; wall {wall:.2f} us per iteration (iterations 51-80, unprofiled)", flush=True)
        k.close()


if __name__ == "__main__":
    main()
