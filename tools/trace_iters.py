"""Per-launch durations of k_expand / k_finish from a rocprofv3 kernel trace, in launch order.

    python tools/trace_iters.py gpurun_out/trace/trace/run_kernel_trace.csv [--kernel k_expand]
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
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_expand")
    a = ap.parse_args()
    rows = load(a.trace)
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if a.kernel in r["Kernel_Name"]]
    d = np.array(d)
    print(f"{a.kernel}: {len(d)} launches, mean {d.mean():.2f} us, median {np.median(d):.2f} us")
    for i in range(0, len(d), 10):
        print(f"  launches {i:4d}-{min(len(d), i + 10) - 1:4d}: " + " ".join(f"{x:6.2f}" for x in d[i:i + 10]))


if __name__ == "__main__":
    main()
