#!/usr/bin/env python3
"""Per-forward conv-kernel time from a rocprofv3 --kernel-trace CSV of bench.py, to check
bench.py's HIP-event `kernel_ms_per_forward`:  trace_per_forward.py TRACE.csv NCONV NFWD
(the last NFWD forwards' NCONV qconv dispatches each; earlier ones are autotune runs)."""
import csv
import json
import sys

path, nconv, nfwd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
q = [r for r in rows if "qconv" in r["Kernel_Name"]][-nconv * nfwd:]
ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in q]
print(json.dumps({"trace": path, "conv_launches_per_forward": nconv, "forwards": nfwd,
                  "conv_ms_per_forward": round(sum(ns) / nfwd / 1e6, 4),
                  "mean_launch_us": round(sum(ns) / len(ns) / 1e3, 2)}))
