"""Per-launch HBM traffic of k_step against the iteration log, fitted per unit of work.

The PMC means of a run mix launches of different sizes (c5's S runs 30k..131k), so the
ratio to the mean algorithmic bytes attributes nothing.  Instead: one rocprofv3 pass per
TCC counter over the same seeded run, then a least-squares fit per launch

    bytes(t) = c0 + cS * S(t) + cA * A(t-1) + cG * nG(t)

(children expanded, children of t-1 inserted, frontier parents) next to the algorithmic
81 B per child + 20 B per frontier node.

On the GPU box:
    python tools/write_attrib.py run c5 131072 60 gpurun_out/wa/log.json        (the run; under rocprofv3 --pmc)
    python tools/write_attrib.py fit gpurun_out/wa/log.json gpurun_out/wa/write gpurun_out/wa/fetch
"""
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(name, samples, n, out):
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
    with open(out, "w") as f:
        json.dump({"workload": name, "samples": samples, "log": log.tolist()}, f)
    k.close()


def counter(dirpath, name):
    """The per-dispatch values of counter `name` for k_step launches, in dispatch order."""
    vals = {}
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and "k_step" in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return np.array([vals[d] for d in sorted(vals)])


def fit(logpath, write_dir, fetch_dir, skip=3):
    L = json.load(open(logpath))
    log = np.array(L["log"], dtype=np.float64)
    S, A, nG = log[:, 5], log[:, 6], log[:, 2]
    Aprev = np.concatenate([[0.0], A[:-1]])
    wr = 1024.0 * counter(write_dir, "WRITE_SIZE")
    rd = 2048.0 * counter(fetch_dir, "FETCH_SIZE")   # gfx950 correction (pmc_summary.py)
    n = min(len(S), len(wr), len(rd))
    print(f"{L['workload']} at {L['samples']} per iteration: {len(S)} iterations, {len(wr)} / {len(rd)} "
          f"k_step dispatches (write / fetch passes); fitting launches {skip}..{n - 1}")
    sl = slice(skip, n)
    X = np.stack([np.ones(n), S[:n], Aprev[:n], nG[:n]], axis=1)[sl]
    alg = 81.0 * S[:n][sl] + 20.0 * nG[:n][sl]
    for nm, y in (("write", wr[:n][sl]), ("read", rd[:n][sl]), ("total", (wr[:n] + rd[:n])[sl])):
        coef, *_ = np.linalg.lstsq(X, y, rcond=None)
        resid = y - X @ coef
        print(f"  {nm:5s} c0 {coef[0] / 1e3:9.1f} KB  cS {coef[1]:7.2f} B/child  cA {coef[2]:8.2f} B/insert  "
              f"cG {coef[3]:8.2f} B/frontier   rms resid {np.sqrt(np.mean(resid ** 2)) / 1e3:8.1f} KB")
    tot = (wr[:n] + rd[:n])[sl]
    print(f"  mean S {S[:n][sl].mean():.0f}  mean traffic {tot.mean() / 1e6:.3f} MB  mean algorithmic "
          f"{alg.mean() / 1e6:.3f} MB  ratio {tot.mean() / alg.mean():.3f}")
    idle = [i for i in range(skip, n) if S[i] == 0]
    busy = [i for i in range(skip, n) if S[i] > 0]
    if busy:
        a_b = 81.0 * S[busy] + 20.0 * nG[busy]
        print(f"  {len(busy)} launches with S > 0: write {wr[busy].mean() / 1e6:.3f} MB, read {rd[busy].mean() / 1e6:.3f} MB "
              f"against algorithmic {a_b.mean() / 1e6:.3f} MB (writes 57 B/child: {57.0 * S[busy].mean() / 1e6:.3f}, "
              f"reads 24 B/child + 20 B/frontier: {(24.0 * S[busy] + 20.0 * nG[busy]).mean() / 1e6:.3f}); ratio "
              f"{(wr[busy] + rd[busy]).mean() / a_b.mean():.3f}")
    if idle:   # launches that expand nothing: what every launch reads whatever its S
        print(f"  {len(idle)} launches with S = 0: write {wr[idle].mean() / 1e3:.1f} KB, read {rd[idle].mean() / 1e3:.1f} KB; "
              f"the RNG state of every slot (24 B x {L['samples']}, loaded at entry before the plan) = "
              f"{24.0 * L['samples'] / 1e3:.1f} KB")
    print("   t        S      A(t-1)   nG    write KB   read KB   algorithmic KB")
    for i in range(skip, n):
        print(f"  {int(log[i, 0]):3d} {int(S[i]):8d} {int(Aprev[i]):8d} {int(nG[i]):6d} {wr[i] / 1e3:10.1f} "
              f"{rd[i] / 1e3:9.1f} {(81.0 * S[i] + 20.0 * nG[i]) / 1e3:10.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    else:
        fit(sys.argv[2], sys.argv[3], sys.argv[4])
