"""Consecutive k_step launches in a rocprofv3 kernel trace: spans, gaps and end-to-end spacing.

    python tools/overlap_trace.py <trace dir or *_kernel_trace.csv> [--kernel k_step] [--first N] [--last N]

For each launch i (dispatch order): its queue, span (end - start), start relative to the
previous launch's end (negative = dispatched while the previous one still ran, the
overlapped form of DESIGN.md §5.6), and end-to-end spacing (end_i - end_{i-1}: the
iteration's cost on the device, whatever the form).  Summary: medians over the rows.
"""
import argparse
import csv
import glob
import os

import numpy as np


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0) or int(r["Start_Timestamp"]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--first", type=int, default=0, help="skip this many launches of the kernel")
    ap.add_argument("--last", type=int, default=0, help="keep only the last N launches (0: all)")
    a = ap.parse_args()
    rows = [r for r in load(a.trace) if a.kernel in r["Kernel_Name"]]
    rows = rows[a.first:]
    if a.last:
        rows = rows[-a.last:]
    st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.float64) / 1e3
    en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.float64) / 1e3
    q = [r.get("Queue_Id", "?") for r in rows]
    print(f"{a.kernel}: {len(rows)} launches")
    print(f"{'i':>4} {'queue':>6} {'span':>8} {'start-prevEnd':>14} {'end-prevEnd':>12} {'start-prevStart':>16}")
    for i in range(len(rows)):
        d0 = st[i] - en[i - 1] if i else float("nan")
        d1 = en[i] - en[i - 1] if i else float("nan")
        d2 = st[i] - st[i - 1] if i else float("nan")
        print(f"{i:4d} {q[i]:>6} {en[i] - st[i]:8.2f} {d0:14.2f} {d1:12.2f} {d2:16.2f}")
    if len(rows) > 1:
        print(f"median span {np.median(en - st):.2f} us, start - prev end {np.median(st[1:] - en[:-1]):.2f} us, "
              f"end - prev end {np.median(en[1:] - en[:-1]):.2f} us, start - prev start {np.median(st[1:] - st[:-1]):.2f} us")


if __name__ == "__main__":
    main()
