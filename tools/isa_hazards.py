"""Scan the gfx950 code objects of a HIP shared library for the VMEM store-data hazard.

    python tools/isa_hazards.py [cudasbmp_amd/libsbmp.so]      (exit 1 if any hazard)

A VMEM store of more than 8 bytes (dwordx3 / dwordx4, cmpswap_x2) reads its data VGPRs
after issue, so a VALU write of one of them needs one wait state in between (CDNA ISA,
"manually inserted wait states").  The compiler pads its own stores with s_nop, but
ROCm 7.2's hazard recognizer skips MUBUF stores whose soffset is an SGPR: round 3 got
`buffer_store_dwordx4 v[8:11], ..., s12` followed by `v_mov_b32 v8, ...`, and the store
wrote the new value.  Every buffer store in kgmt_device.h keeps soffset
0; this scan checks the built library rather than the convention.

Method: the .hip_fatbin section holds one clang offload bundle per translation unit;
each gfx950 code object is unbundled (clang-offload-bundler) and disassembled
(llvm-objdump), and each wide store is checked against the instruction after it.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# stores (and atomics) whose data operand is wider than 8 bytes
WIDE_STORE = re.compile(r"^(buffer|global|flat|scratch)_(store_dwordx[34]|store_b(96|128)|atomic_cmpswap_x2\w*)\b")
VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def vgpr_range(tok: str):
    """(lo, hi) of a VGPR operand token, or None."""
    m = VREG.match(tok)
    if not m:
        return None
    if m.group(1) is not None:
        n = int(m.group(1))
        return n, n
    return int(m.group(2)), int(m.group(3))


def parse(line: str):
    """(mnemonic, [operands]) of one disassembly line (comments stripped), or None."""
    s = line.split("//")[0].strip()
    if not s or s.endswith(":") or s.startswith("."):
        return None
    parts = s.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def scan_lines(lines):
    """Hazards in a sequence of disassembly lines: [(store line, next line)]."""
    insts = [p for p in (parse(l) for l in lines) if p is not None]
    raw = [l.split("//")[0].strip() for l in lines if parse(l) is not None]
    bad = []
    for k, (op, ops) in enumerate(insts[:-1]):
        if not WIDE_STORE.match(op) or not ops:
            continue
        # buffer_store_dwordx4 vdata, vaddr, srsrc, soffset; global_store_dwordx4 vaddr, vdata, saddr
        flat = op.startswith(("global_", "flat_", "scratch_"))
        data = vgpr_range(ops[1]) if flat and len(ops) > 1 else None if flat else vgpr_range(ops[0])
        if data is None:
            continue
        nop, nops = insts[k + 1]
        if nop == "s_nop" or not nop.startswith("v_") or not nops:
            continue
        dst = vgpr_range(nops[0])
        if dst is not None and dst[0] <= data[1] and data[0] <= dst[1]:
            bad.append((raw[k], raw[k + 1]))
    return bad


def code_objects(lib: str, tmp: str):
    """Paths of the gfx950 code objects bundled in lib's .hip_fatbin section."""
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib,
                    os.path.join(tmp, "stripped.so")], check=True, capture_output=True)
    data = open(fat, "rb").read()
    offs = []
    i = data.find(MAGIC)
    while i >= 0:
        offs.append(i)
        i = data.find(MAGIC, i + 1)
    out = []
    for n, (a, b) in enumerate(zip(offs, offs[1:] + [len(data)])):
        bundle = os.path.join(tmp, f"b{n}.bin")
        with open(bundle, "wb") as f:
            f.write(data[a:b])
        co = os.path.join(tmp, f"co{n}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                            f"--input={bundle}", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def scan_library(lib: str):
    """(number of code objects, wide stores seen, hazards) of a built library."""
    with tempfile.TemporaryDirectory() as tmp:
        cos = code_objects(lib, tmp)
        hazards, stores = [], 0
        for co in cos:
            r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                               capture_output=True, text=True)
            lines = r.stdout.splitlines()
            stores += sum(1 for l in lines if (p := parse(l)) and WIDE_STORE.match(p[0]))
            hazards += scan_lines(lines)
        return len(cos), stores, hazards


def kernel_resources(lib: str):
    """{kernel symbol: (vgpr_count, sgpr spill count, private segment bytes)} from the
    code objects' metadata notes."""
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            for b in notes.split("- .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", b)
                vgpr = re.search(r"\.vgpr_count:\s+(\d+)", b)
                priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", b)
                vsp = re.search(r"\.vgpr_spill_count:\s+(\d+)", b)
                if name and vgpr and priv:
                    out[name.group(1)] = (int(vgpr.group(1)), int(vsp.group(1)) if vsp else 0, int(priv.group(1)))
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "cudasbmp_amd",
                                                              "libsbmp.so")
    n, stores, hz = scan_library(lib)
    print(f"{lib}: {n} code objects, {stores} wide stores, {len(hz)} hazards")
    for s, t in hz:
        print(f"  {s}\n    -> {t}")
    sys.exit(1 if hz else 0)


if __name__ == "__main__":
    main()
