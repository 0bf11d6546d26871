"""Static instruction counts of one kernel per source line, from a -gline-tables-only ISA dump.

    hipcc ... -S --cuda-device-only -gline-tables-only kgmt_kernels.hip -o kg.s
    python tools/isa_lines.py kg.s <mangled kernel name> [--top N]

Each instruction is charged to the innermost source line of its .loc directive; the
VALU / SALU / LDS / VMEM split shows where a kernel's instruction budget sits.
"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 60
    files = {}
    cnt = collections.defaultdict(lambda: collections.Counter())
    inside = False
    loc = ("?", 0)
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if line.startswith(name + ":"):
            inside = True
            continue
        if not inside:
            continue
        if line.startswith("\t.size\t" + name) or line.strip() == "s_endpgm" and False:
            break
        m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', line)
        if m:
            loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        m = re.match(r'\t([a-z_0-9]+)', line)
        if not m or line.startswith("\t."):
            continue
        op = m.group(1)
        cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith("s_load")
               and not op.startswith("s_waitcnt") and not op.startswith("s_buffer") else
               "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else
               "smem" if op.startswith(("s_load", "s_buffer")) else "wait" if op.startswith("s_waitcnt") else "other")
        cnt[loc][cls] += 1
        if "s_endpgm" in line:
            pass
    tot = collections.Counter()
    for v in cnt.values():
        tot.update(v)
    print("total", dict(tot))
    rows = sorted(cnt.items(), key=lambda kv: -(kv[1]["valu"] + kv[1]["salu"]))
    for (f, l), c in rows[:top]:
        print(f"{f}:{l:<5} valu {c['valu']:4d} salu {c['salu']:4d} lds {c['lds']:3d} vmem {c['vmem']:3d} smem {c['smem']:3d}")


if __name__ == "__main__":
    main()
