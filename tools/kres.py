#!/usr/bin/env python3
"""Per-kernel resource summary from a hipcc -S (gfx950) listing: VGPR/AGPR/SGPR, spills, LDS."""
import re
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in txt.split("  - .agpr_count:")[1:]:
    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    agpr = blk.split("\n", 1)[0].strip()
    name = g("name")
    if pat not in name:
        continue
    print(f"{name[:70]:70s} vgpr={g('vgpr_count'):>4} agpr={agpr:>3} sgpr={g('sgpr_count'):>4} "
          f"spill={g('vgpr_spill_count')}/{g('sgpr_spill_count')} scratch={g('private_segment_fixed_size')}")
