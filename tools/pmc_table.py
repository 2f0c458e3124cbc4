#!/usr/bin/env python3
"""Per-launch PMC counters of the last engine forward (eager launches of tools/layer_table.py
run --eager), from one or more rocprofv3 --pmc output directories.

    python tools/pmc_table.py META.json DIR [DIR ...] [--json OUT]
Prints one row per launch with every counter collected (summed over the dispatch's XCDs /
instances as rocprofv3 reports them), plus derived ratios when present:
VALU and MFMA instructions per wave, MFMA busy fraction, LDS bank-conflict fraction.
"""
import argparse
import collections
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("meta")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    L = json.load(open(a.meta))["launches"]
    n = len(L)
    per = collections.defaultdict(dict)  # counter -> dispatch id -> value
    names = {}
    for d in a.dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if not r["Kernel_Name"].startswith(("void qnn::", "qnn::")):
                    continue
                did = int(r["Dispatch_Id"])
                per[r["Counter_Name"]][did] = per[r["Counter_Name"]].get(did, 0.0) + float(r["Counter_Value"])
                names[(d, did)] = r["Kernel_Name"]
    rows = []
    for cn, vals in per.items():
        ids = sorted(vals)[-n:]
        for i, did in enumerate(ids):
            if len(rows) <= i:
                rows.append({"i": i, "kernel": L[i]["kernel"], "shape": L[i]["shape"]})
            rows[i][cn] = vals[did]
    for r in rows:
        w = r.get("SQ_WAVES")
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_SALU"):
                if k in r:
                    r[k.replace("SQ_INSTS_", "") + "/wave"] = round(r[k] / w, 1)
        if r.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in r:
            r["mfma_busy"] = round(r["SQ_VALU_MFMA_BUSY_CYCLES"] / r["SQ_BUSY_CYCLES"], 3)
        if r.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in r:
            r["lds_conflict"] = round(r["SQ_LDS_BANK_CONFLICT"] / r["SQ_LDS_IDX_ACTIVE"], 3)
    keys = [k for k in ("VALU/wave", "MFMA/wave", "LDS/wave", "VMEM_RD/wave", "VMEM_WR/wave", "SALU/wave",
                        "mfma_busy", "lds_conflict", "SQ_WAVES") if any(k in r for r in rows)]
    print("i  kernel                     " + " ".join(f"{k:>12s}" for k in keys))
    for r in rows:
        print(f"{r['i']:2d} {r['kernel'][:26]:26s} " + " ".join(f"{r.get(k, float('nan')):12.3f}" for k in keys))
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
