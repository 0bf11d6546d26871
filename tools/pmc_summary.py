"""Summarise rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc [--json profiles/pmc_traffic.json]

Per kernel: mean of every counter over its steady-state dispatches (the first
`--skip` dispatches of each kernel are warm-up).  HBM traffic per launch uses the
gfx950 correction from MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes
of wide coalesced streams, so fetched bytes = 2 * FETCH_SIZE KiB; WRITE_SIZE is
exact for 16-B-per-lane stores.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

import numpy as np


def load(dirpath):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values by dispatch]
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        by_disp = defaultdict(dict)
        names = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        for d in sorted(by_disp):
            for k, v in by_disp[d].items():
                per[names[d]][k].append(v)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=25)
    ap.add_argument("--stat", choices=("median", "mean"), default="median",
                    help="mean: for runs whose launches differ in size (c5), so that counts per child "
                         "match the bench's mean S over the same launches")
    ap.add_argument("--json", default=None)
    ap.add_argument("--samples-per-launch", type=float, default=None,
                    help="children per k_expand / k_step launch in the profiled run (for bytes/child)")
    a = ap.parse_args()
    summary = {}
    subs = [x for x in ("sq", "sq2", "fetch", "write") if os.path.isdir(os.path.join(a.dir, x))] or [""]
    for sub in subs:   # the passes of tools/profile_pmc.sh, or one pass's directory
        for kern, ctrs in load(os.path.join(a.dir, sub)).items():
            short = kern.split("(")[0].replace("void ", "").replace("sbmp::", "")
            for c, vals in ctrs.items():
                v = np.array(vals[a.skip:] if len(vals) > a.skip + 3 else vals)
                summary.setdefault(short, {})[c] = float(np.median(v) if a.stat == "median" else np.mean(v))
                summary[short]["dispatches"] = float(len(v))
    for k, cs in summary.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {v:16.1f}")
    if a.json:
        out = {}
        for k, cs in summary.items():
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                cs.pop("dispatches", None)
                rd = 2.0 * cs["FETCH_SIZE"] * 1024.0
                wr = cs["WRITE_SIZE"] * 1024.0
                key = "k_expand" if k.startswith("k_expand") else "k_step" if k.startswith("k_step") else k
                out[key] = {"kernel": k, "fetch_size_kib": cs["FETCH_SIZE"], "write_size_kib": cs["WRITE_SIZE"],
                            "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                            "correction": "read = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM)"}
                if key in ("k_expand", "k_step") and a.samples_per_launch:
                    out[key]["hbm_bytes_per_child"] = (rd + wr) / a.samples_per_launch
                    # instruction counts for bench.py's valu_frac / salu_frac / wait_frac
                    if "SQ_INSTS_VALU" in cs and "SQ_WAVES" in cs:
                        out[key]["valu_insts_per_child"] = cs["SQ_INSTS_VALU"] / a.samples_per_launch
                        out[key]["salu_insts_per_child"] = cs["SQ_INSTS_SALU"] / a.samples_per_launch
                        out[key]["valu_insts_per_wave"] = cs["SQ_INSTS_VALU"] / cs["SQ_WAVES"]
                        out[key]["salu_insts_per_wave"] = cs["SQ_INSTS_SALU"] / cs["SQ_WAVES"]
                    if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
                        out[key]["wait_any_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
