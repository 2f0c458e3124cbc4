#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc results (rocpd .db) per kernel: mean counter value per
dispatch, plus derived per-wave figures.  usage: pmc_summary.py DIR [DIR...] [--match qconv]"""
import glob
import sqlite3
import sys
from collections import defaultdict

match = "qconv"
args = [a for a in sys.argv[1:]]
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
for root in args:
    vals = defaultdict(lambda: defaultdict(list))
    info = {}
    for f in sorted(glob.glob(f"{root}/**/*.db", recursive=True)):
        con = sqlite3.connect(f)
        q = ("select kernel_name, dispatch_id, counter_name, value, duration, grid_size, workgroup_size, "
             "vgpr_count, accum_vgpr_count, lds_block_size from counters_collection")
        for kn, did, cn, v, dur, grid, wg, vg, ag, lds in con.execute(q):
            if match not in kn:
                continue
            k = kn.split("(")[0][:40] + f" grid={grid}"
            vals[k][cn].append(v)
            info[k] = (grid // wg, wg, vg, ag, lds)
    print("==", root)
    for k, cs in vals.items():
        blocks, wg, vg, ag, lds = info[k]
        waves = blocks * wg // 64
        print(f"  {k}  blocks={blocks} vgpr={vg} agpr={ag} lds={lds}")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c, v in sorted(m.items()):
            print(f"    {c:28s} {v:16.0f}   per-wave {v / waves:10.1f}")
        if "SQ_WAVE_CYCLES" in m:
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"    {c} / WAVE_CYCLES = {m[c] / wc:.3f}")
