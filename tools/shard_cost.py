"""Per-rank kernel costs of the sharded data flow at bench scale, on one GPU: a
local shard group of P virtual ranks with P x 262,144 children per iteration (the
weak-scaling bench at N = P), so every rank's k_finish sees P x 1024 global
blocks.  The ranks run one after another on one stream, so only the per-kernel
means are meaningful, not the wall time.  python tools/shard_cost.py [P ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cudasbmp_amd import KGMT, DeviceBuffer, read_obstacles_csv  # noqa: E402


def main():
    obs = read_obstacles_csv(os.path.join(ROOT, "configurations", "obstacles", "obstacles.csv"))
    d_obs = DeviceBuffer(obs)
    for P in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
        k = KGMT(20.0, 20.0, 16, 8, 60, 1 << 24, 10, 1.0, 0.0, samplesPerIteration=262144 * P, batchRule="fill",
                 fixGNewClear=True, _local_group=P if P > 1 else 0)
        k.begin((5, 5, 0, 0, 0, 0, 0), (2, 18, 0, 0, 0, 0, 0), d_obs, len(obs), 20240807)
        k.enqueue(20)
        k.sync()
        k.set_profiling(True)
        k.reset_kernel_stats()
        k.enqueue(30)
        k.sync()
        st = k.kernel_stats()
        print(f"P={P} (rank 0): " + ", ".join(f"{n} {1e3 * ms / max(1, c):.2f} us x{c}" for n, (c, ms) in st.items()),
              flush=True)
        k.close()


if __name__ == "__main__":
    main()
