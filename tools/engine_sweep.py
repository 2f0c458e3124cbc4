#!/usr/bin/env python3
"""Every tile configuration of every contraction of one engine forward, timed in place.

Builds bench.py's model and an autotuned qnn.Engine (which times each configuration built
for each contraction on the launch stream, HIP events, Engine.tune_table) and prints, per
contraction: its GEMM shape, epilogue kind, the fastest configurations with their kernel
family, and the chosen one.  --json writes the whole table.

    python tools/engine_sweep.py --depth 18 --batch 128 [--model resnet] [--top 6] [--json out.json]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "quantized.pytorch_amd")]


def epi_kind(e):
    """The epilogue kind the library dispatches on (qconv_common.h epi_kind)."""
    if e.mode == 0:
        return "nchw"
    if e.lut:
        return "lut"
    if e.out_bncode and not e.out_f32 and not e.out_code0 and not e.out_code1:
        return "bncode"
    return "gen"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--json")
    a = ap.parse_args()
    import torch
    import bench
    from qnn import _lib
    from qnn.engine import Engine
    dev = torch.device("cuda:0")
    _lib.load()
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch, graph=False)
    rows = []
    for n, ((idx, d, e), times) in enumerate(zip(eng.convs, eng.tune_table)):
        meta = eng.launch_meta[idx]
        best = sorted(times.items(), key=lambda t: t[1])
        kind = epi_kind(e)
        rows.append({"conv": n, "launch": idx, "shape": meta["shape"], "ops": meta["ops"], "bytes": meta["bytes"],
                     "epi": kind, "chosen": eng.tiles[n][0],
                     "us": {str(k): round(ms * 1e3, 2) for k, ms in best}})
        top = ", ".join(f"{k}:{_lib.tile_kernel(k).replace('qconv_', '').replace('_kernel', '')} {ms * 1e3:.1f}"
                        for k, ms in best[:a.top])
        print(f"{n:2d} {str(meta['shape']):24s} {kind:6s} {top}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"model": bench.model_name(a.model, a.depth), "batch": a.batch, "convs": rows}, f, indent=1)


if __name__ == "__main__":
    main()
