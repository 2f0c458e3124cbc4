#!/usr/bin/env python3
"""Per-launch durations of the engine's forward from a rocprofv3 --kernel-trace CSV of
bench.py (the last NFWD graph replays; earlier dispatches are autotune and warm-up):
    forward_breakdown.py TRACE.csv LAUNCHES_PER_FORWARD NFWD [--json out.json]
Prints position, kernel, mean / min us over the replays, and the per-forward total."""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("launches", type=int)
ap.add_argument("nfwd", type=int)
ap.add_argument("--json")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
q = [r for r in rows if r["Kernel_Name"].startswith(("void qnn::", "qnn::"))][-a.launches * a.nfwd:]
assert len(q) == a.launches * a.nfwd, f"only {len(q)} qnn dispatches"
out = []
for i in range(a.launches):
    d = [int(q[f * a.launches + i]["End_Timestamp"]) - int(q[f * a.launches + i]["Start_Timestamp"])
         for f in range(a.nfwd)]
    name = q[i]["Kernel_Name"].replace("void qnn::", "").split("(")[0]
    out.append({"i": i, "kernel": name[:100], "us_mean": round(sum(d) / len(d) / 1e3, 2),
                "us_min": round(min(d) / 1e3, 2)})
    print(f"{i:3d} {out[-1]['us_mean']:8.2f} {out[-1]['us_min']:8.2f}  {name[:110]}")
span = [(int(q[(f + 1) * a.launches - 1]["End_Timestamp"]) - int(q[f * a.launches]["Start_Timestamp"])) / 1e3
        for f in range(a.nfwd)]
tot = sum(r["us_mean"] for r in out)
print(f"sum of kernel means {tot:.1f} us; first-start..last-end per forward {sum(span) / len(span):.1f} us")
if a.json:
    json.dump({"trace": a.trace, "launches": out, "kernel_us_sum": round(tot, 1),
               "forward_span_us": round(sum(span) / len(span), 1)}, open(a.json, "w"), indent=1)
