"""PMC summary of k_step for one workload over chosen iterations (per launch, joined to the log).

bench.py's roofline fields (valu_frac, salu_frac, wait_frac, traffic) come from a committed
PMC summary per workload; a bench run mixes warm-up, timed, flush and replayed launches,
whose means attribute nothing when launch sizes differ (c5: S from 0 to 131,072).  This
takes one seeded run of iterations 1..N (every k_step dispatch is one iteration, in order),
one rocprofv3 pass per counter group, and sums the counters over iterations [first, last]:

    per child: SQ_INSTS_VALU, SQ_INSTS_SALU, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, the
               gfx950 correction of MI355X_MICROARCH.md), the algorithmic bytes beside them
    per wave:  SQ_INSTS_VALU, SQ_INSTS_SALU;   wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES

On the GPU box (tools/gpu_cycle.sh wlpmc <out> <workload> <samples> <N> <first> <last>):
    rocprofv3 --pmc <group> -d <out>/<g> -o run --output-format csv -- \
        python3 tools/pmc_workload.py run c5 131072 40 <out>/log.json
    python3 tools/pmc_workload.py sum <out> 6 40 --json profiles/pmc_c5_131072.json
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GROUPS = {"sq": ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES"],
          "fetch": ["FETCH_SIZE"], "write": ["WRITE_SIZE"]}


def per_dispatch(dirpath, kernel="k_step"):
    """{counter: [value per k_step dispatch, in dispatch order]}"""
    per, names = {}, {}
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per.setdefault(d, {})
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    ids = [d for d in sorted(per) if kernel in names[d]]
    out = {}
    for d in ids:
        for c, v in per[d].items():
            out.setdefault(c, []).append(v)
    return out, (names[ids[0]] if ids else kernel)


def run(name, samples, n, path):
    from cudasbmp_amd import DeviceBuffer, read_obstacles_csv
    from cudasbmp_amd.config import workload
    from cudasbmp_amd.kgmt import KGMT
    cfg = workload(name)
    obs = read_obstacles_csv(cfg["obstacles"])
    pl = dict(cfg["planner"])
    pl.update(numIterations=n + 2)
    k = KGMT(**pl, samplesPerIteration=samples, agent=cfg["agent"], batchRule=cfg["batchRule"], fixGNewClear=True)
    d_obs = DeviceBuffer(obs)
    k.begin(cfg["initial"], cfg["goal"], d_obs, len(obs), 20240807)
    k.enqueue(n)
    k.sync()
    log = k.iter_log()[:n]
    with open(path, "w") as f:
        json.dump({"workload": name, "samples": samples, "log": log.tolist(), "path": k.path_info()}, f)
    k.close()


def summarize(out, first, last):
    meta = json.load(open(os.path.join(out, "log.json")))
    log = np.array(meta["log"], dtype=np.float64)   # itr, treeSizeBefore, nG, k, nExp, S, A, treeSizeAfter, goal
    c = {}
    kname = "k_step"
    for g in GROUPS:
        vals, kname = per_dispatch(os.path.join(out, g))
        c.update(vals)
    n = len(log)
    sel = slice(first - 1, last)
    S = log[sel, 5]
    nG = np.minimum(log[sel, 2], log[sel, 5])
    A_prev = log[first - 2:last - 1, 6] if first > 1 else np.concatenate([[0.0], log[:last - 1, 6]])
    tot = {k: float(np.sum(np.array(v[:n])[sel])) for k, v in c.items()}
    nS = float(S.sum())
    hbm = 2.0 * tot["FETCH_SIZE"] * 1024.0 + tot["WRITE_SIZE"] * 1024.0
    algo = 81.0 * nS + 20.0 * float(nG.sum()) + 76.0 * float(A_prev.sum())
    res = {"kernel": kname, "workload": meta["workload"], "samples_per_iteration": meta["samples"],
           "iterations": [first, last], "launches": last - first + 1, "mean_S": nS / (last - first + 1),
           "stalled_iterations": int((S == 0).sum()),
           "hbm_bytes_per_child": hbm / nS, "algorithmic_bytes_per_child": algo / nS,
           "traffic_over_algorithmic": hbm / algo,
           "valu_insts_per_child": tot["SQ_INSTS_VALU"] / nS, "salu_insts_per_child": tot["SQ_INSTS_SALU"] / nS,
           "valu_insts_per_wave": tot["SQ_INSTS_VALU"] / tot["SQ_WAVES"],
           "salu_insts_per_wave": tot["SQ_INSTS_SALU"] / tot["SQ_WAVES"],
           "wait_any_frac": tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"],
           "correction": "read = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
           "source": "tools/pmc_workload.py: one rocprofv3 --pmc pass per group, summed over the iterations"}
    return res


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("workload")
    r.add_argument("samples", type=int)
    r.add_argument("n", type=int)
    r.add_argument("path")
    s = sub.add_parser("sum")
    s.add_argument("out")
    s.add_argument("first", type=int)
    s.add_argument("last", type=int)
    s.add_argument("--json", default=None)
    a = ap.parse_args()
    if a.cmd == "run":
        run(a.workload, a.samples, a.n, a.path)
        return
    res = summarize(a.out, a.first, a.last)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"k_step": res}, f, indent=1)


if __name__ == "__main__":
    main()
