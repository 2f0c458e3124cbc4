#!/usr/bin/env python3
"""HBM traffic of the conv launches of one engine forward, from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950) over `profile_engine.py`.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half the bytes of 16-B-per-lane streaming reads
(global_load / global_load_lds dwordx4, the conv kernel's only read width) -> x2;
WRITE_SIZE is exact for 16-B-per-lane stores (the conv epilogue's store width).

    python tools/traffic.py FETCH_DIR WRITE_DIR PROFILE_LOG OUT_JSON [--source TEXT]

PROFILE_LOG is profile_engine.py's per-launch output of the same run (launch order and
algorithmic bytes).  The last `reps` forwards' conv dispatches are averaged (the engine's
autotune runs precede them).
"""
import csv
import glob
import json
import sys


def counter_rows(root, name):
    rows = []
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == name and "qconv" in r["Kernel_Name"]:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    fdir, wdir, plog, out = sys.argv[1:5]
    source = sys.argv[sys.argv.index("--source") + 1] if "--source" in sys.argv else ""
    launches = []
    with open(plog) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("{") and '"kernel": "qnn_qconv2d_fwd"' in line:
                launches.append(json.loads(line))
    n = len(launches)
    fetch = counter_rows(fdir, "FETCH_SIZE")
    write = counter_rows(wdir, "WRITE_SIZE")
    reps = min(len(fetch), len(write)) // n - 1  # drop the autotune + first forward
    reps = max(1, min(reps, 5))
    f_tail, w_tail = fetch[-reps * n:], write[-reps * n:]
    per = []
    for i, L in enumerate(launches):
        fb = sum(2 * 1024 * f_tail[r * n + i][1] for r in range(reps)) / reps
        wb = sum(1024 * w_tail[r * n + i][1] for r in range(reps)) / reps
        per.append({"i": L["i"], "MxNxK": L["MxNxK"], "alg_bytes": L.get("alg_bytes"), "fetch_bytes": round(fb),
                    "write_bytes": round(wb), "hbm_over_alg": round((fb + wb) / L["alg_bytes"], 3)
                    if L.get("alg_bytes") else None, "us": L["us"]})
    tot = sum(p["fetch_bytes"] + p["write_bytes"] for p in per)
    alg = sum(p["alg_bytes"] or 0 for p in per)
    us = sum(p["us"] for p in per)
    res = {"hbm_bytes_per_forward": tot, "alg_bytes_per_forward": alg, "conv_launches": n, "reps": reps,
           "hbm_GBs_over_conv_time": round(tot / (us * 1e-6) / 1e9, 1),
           "source": source or f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({fdir}, {wdir}); FETCH x2 (gfx950)",
           "per_launch": per}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_launch"}))


if __name__ == "__main__":
    main()
