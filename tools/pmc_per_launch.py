"""Per-dispatch SQ counters of one kernel from a rocprofv3 --pmc run, in dispatch order.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
        -d <out> -o run --output-format csv -- python3 tools/iter_times.py 40
    python tools/pmc_per_launch.py <out> [--kernel k_step] [--first N]

With tools/iter_times.py the k step dispatches 1..N are iterations 1..N, so a slow
iteration's VALU and wait counts per wave can be set beside a steady-state one.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--first", type=int, default=40)
    a = ap.parse_args()
    per = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    ids = [d for d in sorted(per) if a.kernel in names[d]][: a.first]
    cols = sorted({c for d in ids for c in per[d]})
    print(f"{a.kernel}: {len(ids)} dispatches; per wave: " + ", ".join(c for c in cols if c != "SQ_WAVES"))
    print("  i  " + " ".join(f"{c.replace('SQ_', ''):>14s}" for c in cols if c != "SQ_WAVES"))
    for i, d in enumerate(ids, 1):
        w = per[d].get("SQ_WAVES", 1.0) or 1.0
        print(f"{i:3d}  " + " ".join(f"{per[d][c] / w:14.1f}" for c in cols if c != "SQ_WAVES"))


if __name__ == "__main__":
    main()
