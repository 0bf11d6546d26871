"""Copy a round's GPU profile (tools/profile_round.sh output) into profiles/<round>/.

    python tools/summarize_round.py gpurun_out/r01 r01 [--bench gpurun_out/b.json]

Writes
  profiles/<round>/kernel_stats.csv        rocprofv3 --kernel-trace --stats of `python bench.py`
  profiles/<round>/bench_under_rocprof.json the bench line of that same profiled command
  profiles/<round>/expand_windows.json     k_expand durations from the kernel trace over the
                                            bench's own windows (warm-up, timed, profiled): the
                                            profiled-window mean is what the bench's roofline
                                            divides by, so the two can be compared directly
  profiles/<round>/pmc_summary.txt         per-kernel counter medians (tools/pmc_summary.py)
  profiles/pmc_traffic.json                HBM bytes per k_expand launch / per child (read by bench.py)
  profiles/<round>/bench.json              an unprofiled bench line, if --bench is given
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("round")
    ap.add_argument("--bench", default=None)
    a = ap.parse_args()
    dst = os.path.join(ROOT, "profiles", a.round)
    os.makedirs(dst, exist_ok=True)
    trace_dir = os.path.join(a.src, "trace")
    shutil.copy(glob.glob(os.path.join(trace_dir, "**", "*kernel_stats.csv"), recursive=True)[0],
                os.path.join(dst, "kernel_stats.csv"))
    bench = json.loads(open(os.path.join(a.src, "bench.json")).read().strip().splitlines()[-1])
    json.dump(bench, open(os.path.join(dst, "bench_under_rocprof.json"), "w"), indent=1)

    rows = list(csv.DictReader(open(glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"),
                                                recursive=True)[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hot = "k_step" if any("k_step" in r["Kernel_Name"] for r in rows) else "k_expand"
    exp = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
           if hot in r["Kernel_Name"]]
    W, K = bench["warmup"], bench["steps"]
    # bench.py: run A = W warm-up + K timed launches; run B (same seed) = W warm-up +
    # K event-stamped launches replaying the timed iterations.
    win = {"warmup": exp[:W], "timed": exp[W:W + K], "replay_warmup": exp[W + K:2 * W + K],
           "replay_timed": exp[2 * W + K:2 * W + 2 * K]}
    out = {name: {"launches": len(v), "mean_us": round(float(np.mean(v)), 3),
                  "median_us": round(float(np.median(v)), 3)} for name, v in win.items() if v}
    out["bench_roofline_avg_launch_us"] = bench["roofline"]["avg_launch_us"]
    out["kernel"] = hot
    out["note"] = (f"{hot} launches in trace order (k_step: the flush passes before read-backs are launches too); the first 2W+2K belong to the bench planner "
                   "(the TTFS demo plans follow).  The bench's roofline divides algorithmic bytes by the mean of "
                   "its own dispatch-stamped HIP events over replay_timed (= the timed iterations).  Under "
                   "rocprofv3 those HIP events read high; compare the unprofiled bench line (bench.json).")
    json.dump(out, open(os.path.join(dst, "expand_windows.json"), "w"), indent=1)

    S = bench["config"]["mean_S"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.join(a.src, "pmc"),
                        "--skip", "20", "--samples-per-launch", str(S),
                        "--json", os.path.join(ROOT, "profiles", "pmc_traffic.json")],
                       capture_output=True, text=True, check=True)
    open(os.path.join(dst, "pmc_summary.txt"), "w").write(r.stdout)
    if a.bench:
        line = open(a.bench).read().strip().splitlines()[-1]
        json.dump(json.loads(line), open(os.path.join(dst, "bench.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
