#!/usr/bin/env python3
"""Per-launch roofline table of one engine forward.

On the GPU box, under rocprofv3 (kernel trace):
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- \\
        python3 tools/layer_table.py run --depth 50 --batch 256 --meta META.json
builds the engine, writes its per-launch metadata (Engine.launch_meta: algorithmic int8
ops, minimum HBM bytes, shape; plus the tile plan) and replays the hipGraph --fwd times.
Then, anywhere:
    python tools/layer_table.py join DIR/run_kernel_trace.csv META.json OUT.json
joins the last --fwd replays' dispatch durations (rocprof, the source of record) with the
metadata: per launch us, TOP/s, GB/s, fraction of the 5 POPS int8 peak, of 8 TB/s HBM,
and of the attainable bound max(ops/peak, bytes/HBM) -- 1.0 = at the roofline.
"""
import argparse
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_TOPS, PEAK_GBS = 5000.0, 8000.0


def run(a):
    sys.path[:0] = [HERE, os.path.join(HERE, "quantized.pytorch_amd")]
    import torch
    import bench
    from qnn import synthetic
    from qnn.engine import Engine
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch)
    eng.input.copy_(synthetic.input_batch((a.batch, 3, 224, 224), 1234).to(dev))
    plans = {i: Engine.plan(d, e) for i, d, e in eng.convs}
    meta = [dict(m, i=i, plan=list(plans[i]) if i in plans else None) for i, m in enumerate(eng.launch_meta)]
    with open(a.meta, "w") as f:
        json.dump({"model": bench.model_name(a.model, a.depth), "batch": a.batch, "fwd": a.fwd,
                   "launches": meta}, f)
    with torch.no_grad():
        for _ in range(a.fwd):
            eng._run_ops() if a.eager else eng()
    torch.cuda.synchronize()


def join(a):
    meta = json.load(open(a.meta))
    L = meta["launches"]
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    q = [r for r in rows if r["Kernel_Name"].startswith(("void qnn::", "qnn::"))][-len(L) * meta["fwd"]:]
    assert len(q) == len(L) * meta["fwd"], f"{len(q)} qnn dispatches for {len(L)} x {meta['fwd']}"
    out = []
    for i, m in enumerate(L):
        ns = [int(q[f * len(L) + i]["End_Timestamp"]) - int(q[f * len(L) + i]["Start_Timestamp"])
              for f in range(meta["fwd"])]
        us = sum(ns) / len(ns) / 1e3
        t_roof = max(m["ops"] / (PEAK_TOPS * 1e12), m["bytes"] / (PEAK_GBS * 1e9)) * 1e6
        out.append({"i": i, "kernel": m["kernel"], "shape": m["shape"], "plan": m["plan"],
                    "dispatch": q[i]["Kernel_Name"].replace("void qnn::", "").split("(")[0][:90],
                    "us": round(us, 2), "ops": m["ops"], "bytes": m["bytes"],
                    "tops": round(m["ops"] / us / 1e6, 1), "gbs": round(m["bytes"] / us / 1e3, 1),
                    "frac_mfma": round(m["ops"] / us / 1e6 / PEAK_TOPS, 4),
                    "frac_hbm": round(m["bytes"] / us / 1e3 / PEAK_GBS, 4),
                    "bound": "mfma" if m["ops"] / PEAK_TOPS / 1e12 >= m["bytes"] / PEAK_GBS / 1e9 else "hbm",
                    "frac_attainable": round(t_roof / us, 4)})
    tot = sum(r["us"] for r in out)
    conv = [r for r in out if r["kernel"] == "qnn_qconv2d_fwd"]
    ops = sum(r["ops"] for r in conv)
    cus = sum(r["us"] for r in conv)
    res = {"source": f"rocprofv3 --kernel-trace, last {meta['fwd']} hipGraph replays ({os.path.basename(a.trace)}); "
                     f"ops/bytes from qnn.Engine.launch_meta",
           "model": meta["model"], "batch": meta["batch"], "kernel_us_per_forward": round(tot, 1),
           "conv_us_per_forward": round(cus, 1), "conv_tops": round(ops / cus / 1e6, 1),
           "conv_frac_mfma": round(ops / cus / 1e6 / PEAK_TOPS, 4), "launches": out}
    json.dump(res, open(a.out, "w"), indent=1)
    for r in out:
        print(f"{r['i']:3d} {r['kernel'][:22]:22s} {r['us']:8.2f}us {r['tops']:7.1f}TOPS {r['gbs']:7.1f}GB/s "
              f"mfma {r['frac_mfma']:.3f} hbm {r['frac_hbm']:.3f} attain {r['frac_attainable']:.3f} {r['shape']}")
    print(json.dumps({k: v for k, v in res.items() if k != "launches"}))


def counter_rows(root, name):
    rows = []
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == name and r["Kernel_Name"].startswith(("void qnn::", "qnn::")):
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return sorted(rows)


def pmc(a):
    """HBM bytes per launch of the last forward(s) from two PMC passes (MI355X_MICROARCH.md,
    HBM section: FETCH_SIZE / WRITE_SIZE in KiB; gfx950 FETCH_SIZE counts half the bytes of
    16-B-per-lane streaming reads -> x2; WRITE_SIZE exact for 16-B stores)."""
    meta = json.load(open(a.meta))
    L = meta["launches"]
    n = len(L)
    fetch, write = counter_rows(a.fetch, "FETCH_SIZE"), counter_rows(a.write, "WRITE_SIZE")
    k = min(len(fetch), len(write)) // n
    assert k >= 1, f"{len(fetch)} / {len(write)} counter rows for {n} launches"
    k = min(k, meta["fwd"])
    per = []
    for i, m in enumerate(L):
        fb = sum(2 * 1024 * fetch[len(fetch) - (f + 1) * n + i][1] for f in range(k)) / k
        wb = sum(1024 * write[len(write) - (f + 1) * n + i][1] for f in range(k)) / k
        per.append({"i": i, "kernel": m["kernel"], "shape": m["shape"], "alg_bytes": m["bytes"],
                    "fetch_bytes": round(fb), "write_bytes": round(wb),
                    "hbm_over_alg": round((fb + wb) / m["bytes"], 3) if m["bytes"] else None})
    tot = sum(p["fetch_bytes"] + p["write_bytes"] for p in per)
    conv = [p for p in per if p["kernel"] == "qnn_qconv2d_fwd"]
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({a.fetch}, {a.write}); FETCH x2 (gfx950), "
                     "KiB -> bytes; eager launches of tools/layer_table.py run",
           "model": meta["model"], "batch": meta["batch"], "forwards_averaged": k,
           "hbm_bytes_per_forward": tot, "alg_bytes_per_forward": sum(p["alg_bytes"] for p in per),
           "conv_hbm_bytes_per_forward": sum(p["fetch_bytes"] + p["write_bytes"] for p in conv),
           "conv_alg_bytes_per_forward": sum(p["alg_bytes"] for p in conv), "launches": per}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k_: v for k_, v in res.items() if k_ != "launches"}))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--depth", type=int, default=50)
    r.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    r.add_argument("--batch", type=int, default=256)
    r.add_argument("--fwd", type=int, default=10)
    r.add_argument("--meta", required=True)
    r.add_argument("--eager", action="store_true", help="eager launches (PMC passes) instead of graph replays")
    pm = sub.add_parser("pmc")
    pm.add_argument("fetch")
    pm.add_argument("write")
    pm.add_argument("meta")
    pm.add_argument("out")
    j = sub.add_parser("join")
    j.add_argument("trace")
    j.add_argument("meta")
    j.add_argument("out")
    a = ap.parse_args()
    {"run": run, "join": join, "pmc": pmc}[a.cmd](a)


if __name__ == "__main__":
    main()
