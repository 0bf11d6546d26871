"""Phase timeline of one k_expand launch from s_memrealtime stamps (100 MHz).

    SBMP_TIMELINE_ITER=40 SBMP_TIMELINE_OUT=gpurun_out/tl.bin python bench.py ...
    python tools/timeline.py gpurun_out/tl.bin
    python tools/timeline.py gpurun_out/tl.bin.fin      # k_finish of the same iteration

Stamps per wave (cudasbmp_amd/csrc/kgmt_kernels.hip, k_expand): 0 entry, 1 after the
LDS prologue barrier, 2 after propagation, 3 after accept + slot stores, 4 after region
aggregation, 5 after the flush barrier, 6 end of the counter flush.
"""
import sys

import numpy as np

NAMES = ["entry", "prologue", "propagate", "accept+store", "count_regions", "barrier", "flush"]
# k_step (SBMP_STEP=1, the default on one rank): 1 after the count scan, 2 after the
# parent/insert/prefetch loads are issued, 3 after propagation, 4 after the hand-off check
# (a build with -DSBMP_TL_PROLOGUE as well moves stamp 4 to the plan's barrier and stamp 5
# to the located parent, splitting scan -> issued)
STEP_NAMES = ["entry", "scan", "issued", "propagate", "handoff", "barrier", "end"]


FIN_PLAN = ["entry", "prefix", "deltas", "r2new", "cov", "scores", "R1Score", "end"]
FIN_INSERT = ["entry", "loads", "prefix", "insert", "-", "-", "-", "end"]


def finish(path):
    """k_finish stamps (<out>.fin): block 0 = plan_iteration, blocks 1.. = insert_block."""
    a = np.fromfile(path, dtype=np.int64).reshape(-1, 8)
    t0 = a[a[:, 0] != 0, 0].min()
    us = np.where(a != 0, (a - t0) / 100.0, np.nan)
    print("plan_iteration (block 0): " + "  ".join(f"{n} {us[0, i]:.2f}" for i, n in enumerate(FIN_PLAN)
                                                   if not np.isnan(us[0, i])))
    ins = us[1:]
    live = ~np.isnan(ins[:, 7])
    print(f"insert blocks: {live.sum()} stamped")
    print("stamp           p10     p50     p90     max")
    for i, n in enumerate(FIN_INSERT):
        col = ins[live, i]
        col = col[~np.isnan(col)]
        if len(col):
            print(f"  {n:10s} " + " ".join(f"{x:7.2f}" for x in np.percentile(col, [10, 50, 90, 100])) + f"  (n={len(col)})")


def main():
    global NAMES
    if sys.argv[1].endswith(".fin"):
        finish(sys.argv[1])
        return
    a = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 8)
    if "--step" in sys.argv:   # k_step: the planner's entry / publish stamps are in <out>.fin[0:2]
        NAMES = STEP_NAMES
        f = np.fromfile(sys.argv[1] + ".fin", dtype=np.int64)
        t0w = a[a[:, 6] != 0, 0].min()
        print(f"planner: entry {(f[0] - t0w) / 100.0:+.2f} us, publish {(f[1] - t0w) / 100.0:+.2f} us "
              f"(relative to the first expanding wave's entry)")
        ex = f[8:8 + 64].reshape(8, 8)   # k_oneshot of the same iteration (sharded ranks), one row per chunk
        if (ex[:, 0] != 0).any():
            t_end = a[a[:, 6] != 0, 6].max()
            print("exchange (k_oneshot chunks, or the fused workers; us after the last k_step wave's end):  entry  stored  mirror  fenced  "
                  "flags   end")
            for c in range(8):
                if ex[c, 0]:
                    print(f"  chunk {c}                                                " +
                          " ".join(f"{(ex[c, i] - t_end) / 100.0:7.2f}" for i in range(6)))
    live = a[a[:, 6] != 0]
    print(f"{len(a)} waves, {len(live)} ran the full path")
    t0 = live[:, 0].min()
    us = (live[:, :7] - t0) / 100.0
    print("stamp              p0      p10     p50     p90     max   (us since first wave entry)")
    for i, n in enumerate(NAMES):
        q = np.percentile(us[:, i], [0, 10, 50, 90, 100])
        print(f"  {i} {n:14s} " + " ".join(f"{x:7.2f}" for x in q))
    print("phase durations per wave (us):  p10     p50     p90")
    for i in range(1, 7):
        dd = us[:, i] - us[:, i - 1]
        q = np.percentile(dd, [10, 50, 90])
        print(f"  {NAMES[i - 1]:>14s} -> {NAMES[i]:14s} " + " ".join(f"{x:7.2f}" for x in q))
    hw = live[:, 7] & 0xffffffff
    xcc = (live[:, 7] >> 32) & 0xf
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xf
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
    ends = us[:, 6]
    uk, inv = np.unique(key, return_inverse=True)
    per_max = np.array([ends[inv == i].max() for i in range(len(uk))])
    per_n = np.bincount(inv)
    print(f"SIMDs used {len(uk)}, waves per SIMD: min {per_n.min()} median {np.median(per_n)} max {per_n.max()}")
    print("last wave end per SIMD (us): p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(per_max, [10, 50, 90, 100])))
    for n_ in sorted(set(per_n.tolist())):
        m = per_n == n_
        print(f"  SIMDs with {n_} waves: {m.sum():4d}, last end p50 {np.median(per_max[m]):.2f} max {per_max[m].max():.2f}")
    blk = np.arange(len(a))[a[:, 6] != 0] // 4
    for x in range(8):
        m = (blk % 8) == x
        if m.any():
            print(f"  blockIdx%8=={x}: entry p50 {np.median(us[m, 0]):6.2f}  end p50 {np.median(us[m, 6]):6.2f}  "
                  f"end max {us[m, 6].max():6.2f}")


if __name__ == "__main__":
    main()
