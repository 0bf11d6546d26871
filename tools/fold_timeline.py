"""Phase timeline of one k_fold_r2 iteration's workgroups from a -DSBMP_TIMELINE build.

    SBMP_TIMELINE_ITER=<t> SBMP_TIMELINE_OUT=gpurun_out/f.bin python3 bench.py ...   (t inside the folded window)
    python3 tools/fold_timeline.py gpurun_out/f.bin.fin

Stamps per wave (k_fold_r2): 0 entry, 1 control block read + histogram clear issued,
2 after the clear barrier, 3 key loads landed, 4 adds issued, 5 after the add barrier,
6 flush atomics complete; 7 = XCC id << 32 | HW_ID.  Microseconds from the earliest entry.
"""
import sys

import numpy as np

NAMES = ["entry", "clear", "barrier1", "keys", "adds", "barrier2", "flush"]


def main():
    a = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 8)[9:]   # rows 0-8: k_step's planner and exchange
    live = a[:, 6] != 0
    a = a[live]
    t0 = a[:, 0].min()
    us = (a[:, :7] - t0) / 100.0
    print(f"{len(a)} waves stamped")
    print("stamp          p10     p50     p90     max")
    for i, n in enumerate(NAMES):
        print(f"  {n:10s} " + " ".join(f"{x:7.2f}" for x in np.percentile(us[:, i], [10, 50, 90, 100])))
    d = np.diff(us, axis=1)
    print("phase (per wave)   p50     max")
    for i in range(6):
        print(f"  {NAMES[i]}->{NAMES[i + 1]:9s} {np.percentile(d[:, i], 50):7.2f} {d[:, i].max():7.2f}")


if __name__ == "__main__":
    main()
