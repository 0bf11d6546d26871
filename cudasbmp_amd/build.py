"""Build libsbmp.so (HIP kernels for gfx950 + the C ABI) in-tree with hipcc.

    python -m cudasbmp_amd.build [--force] [--verbose]

The shared library lands next to this file (cudasbmp_amd/libsbmp.so) so it
travels with the repository snapshot to the GPU box.  Objects are rebuilt only
when a source or header is newer than the object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "_obj")
LIB = os.path.join(PKG, "libsbmp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SBMP_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off + explicit fmaf: the kernels and the CPU oracle execute the
# same float operation sequence.  Correctly rounded fp32
# division/sqrt match the oracle's IEEE operations.
COMMON = [
    "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    # The SLP vectoriser packs the per-obstacle hit bits of the Euler step into
    # 16-bit integer vectors (~25 extra VALU per step); float pairs that should be
    # packed are written as float2 by hand (kgmt_device.h sincos_poly2).
    "-fno-slp-vectorize",
    # The first 16 kernel-argument dwords arrive preloaded in SGPRs (gfx950): k_step's
    # first loads issue without a scalar round trip to the kernel-argument segment.
    "-mllvm", "-amdgpu-kernarg-preload-count=16",
    f"--offload-arch={ARCH}",
    "-I", os.path.join(ROOT, "include"), "-I", CSRC,
    "-Wall", "-Wno-unused-result",
]
# Extra compile flags for experiments (e.g. scheduler strategies in an A/B variant).
EXTRA = os.environ.get("SBMP_HIPCC_FLAGS", "").split()
LINK = ["-shared", f"--offload-arch={ARCH}", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "sbmp", "*.h")))


def _compile(src: str, force: bool, verbose: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + COMMON + EXTRA + lang + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC] + objs + LINK + ["-o", LIB]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    main()
