#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a hipcc -S listing (MFMA / VALU / LDS /
SALU / VMEM), and the VALU mix of the blocks that hold MFMAs: a quick look at a hot loop.
  python tools/isa_blocks.py kernel.s NAME_SUBSTRING [--min-valu 40]"""
import collections
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
minv = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[3] == "--min-valu" else 40
s = open(src).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, flags=re.M) if pat in m.group(1)]
for name in names:
    i = s.find(name + ":")
    j = s.find(".Lfunc_end", i)
    blocks, cur = [], None
    for line in s[i:j].split("\n"):
        m = re.match(r"^(\.LBB\S+):", line)
        if m:
            cur = [m.group(1), collections.Counter()]
            blocks.append(cur)
            continue
        if cur is None or not line.strip():
            continue
        op = line.strip().split()[0]
        k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_")
             else "salu" if op.startswith("s_") else "vmem" if op.startswith(("global_", "buffer_")) else None)
        if k:
            cur[1][k] += 1
            if k == "valu":
                cur[1]["op:" + op] += 1
    print(name[:110])
    for b, c in blocks:
        if c["mfma"] or c["valu"] >= minv:
            print(f"  {b}: mfma {c['mfma']} valu {c['valu']} lds {c['lds']} salu {c['salu']} vmem {c['vmem']}")
            if c["mfma"]:
                print("    " + ", ".join(f"{k[3:]} {n}" for k, n in c.most_common() if k.startswith("op:")))
