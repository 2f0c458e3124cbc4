#!/usr/bin/env python3
"""Summarize tools/sweep_tiles.py JSONL output: best qconv.hip vs best qconv16.hip config per layer
(optionally with an ablation run beside it).  python tools/sweep_summary.py sweep.jsonl [ablate.jsonl]"""
import json
import sys
from collections import defaultdict

rows = [json.loads(l) for l in open(sys.argv[1])]
abl = {}
if len(sys.argv) > 2:
    for l in open(sys.argv[2]):
        r = json.loads(l)
        abl[(r["layer"], r["cfg"])] = r["us"]
g = defaultdict(list)
for r in rows:
    g[r["layer"]].append(r)
for L, rs in g.items():
    old = [r for r in rs if r["cfg"] < 18]
    q = [r for r in rs if r["cfg"] >= 18]
    bo = min(old, key=lambda r: r["us"])
    s = f"{L:28s} old {bo['cfg']:2d} {bo['us']:6.1f} {bo['frac']:.3f} [noepi {abl.get((L, bo['cfg']), 0):5.1f}]"
    if q:
        bq = min(q, key=lambda r: r["us"])
        s += f" | q16 {bq['cfg']} {bq['us']:6.1f} {bq['frac']:.3f} :: " + " ".join(
            f"{r['cfg']}:{r['us']:.0f}/{abl.get((L, r['cfg']), 0):.0f}" for r in q)
    neq = [r["cfg"] for r in rs if r["equal_cfg5"] is False]
    print(s, "NEQ" + str(neq) if neq else "")
