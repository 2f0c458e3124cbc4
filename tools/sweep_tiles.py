#!/usr/bin/env python3
"""Time every tile configuration of the int8 contraction on the benchmark layers.

For each layer (SURVEY.md §8(d) shapes at the BASELINE batch sizes) the drop-in
QConv2d forward runs once (quantize + pack + descriptors), then the conv launch
alone is re-issued with each configuration forced (qnn_conv_desc.tile), timed with
HIP events on the launch stream (median of --reps), and its output compared
bitwise with configuration 5's (every configuration computes identical results).

    python tools/sweep_tiles.py [--reps 20] [--only headline] [--json out.jsonl]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "quantized.pytorch_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402
from qnn.quantize import QConv2d  # noqa: E402

PEAK = 5000.0
# name: (cin, cout, k, stride, pad, N, H)
LAYERS = {
    "headline_r50_l3_3x3_256_b256": (256, 256, 3, 1, 1, 256, 14),
    "r50_l4_3x3_512_b256": (512, 512, 3, 1, 1, 256, 7),
    "r50_l1_3x3_64_b256": (64, 64, 3, 1, 1, 256, 56),
    "r50_l2_3x3_128_b256": (128, 128, 3, 1, 1, 256, 28),
    "r50_3x3_s2_256_b256": (256, 256, 3, 2, 1, 256, 28),
    "r18_l1_3x3_64_b128": (64, 64, 3, 1, 1, 128, 56),
    "r18_l2_3x3_128_b128": (128, 128, 3, 1, 1, 128, 28),
    "r18_l2_3x3_s2_64_128_b128": (64, 128, 3, 2, 1, 128, 56),
    "r18_l3_3x3_256_b128": (256, 256, 3, 1, 1, 128, 14),
    "r18_l4_3x3_512_b128": (512, 512, 3, 1, 1, 128, 7),
    "r18_stem_7x7_b128": (3, 64, 7, 2, 3, 128, 224),
    "mbn_stem_3x3_b512": (3, 32, 3, 2, 1, 512, 224),
    "r50_1x1_1024_256_b256": (1024, 256, 1, 1, 0, 256, 14),
    "r50_1x1_64_256_b256": (64, 256, 1, 1, 0, 256, 56),
    "r50_1x1_s2_512_1024_b256": (512, 1024, 1, 2, 0, 256, 28),
    "r18_1x1_s2_64_128_b128": (64, 128, 1, 2, 0, 128, 56),
}


def sweep(name, shape, reps, dev, cfgs=None):
    cin, cout, k, st, pd, N, H = shape
    m = QConv2d(cin, cout, k, stride=st, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 1)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(3.0)
    m.qnn_keep_input = True
    wrap = wrap.to(dev).eval()
    x = torch.randn(N, cin, H, H, device=dev).relu_()
    with torch.no_grad():
        y = wrap(x)
    torch.cuda.synchronize()
    d, e = m._last_conv
    # re-issue the conv launch alone on the forward's own codes and descriptors
    xq_ptr = m._last_xq.data_ptr()
    st_ = _lib.stream_of(y)
    rows = []
    ref = None
    ops = 2 * N * cout * y.shape[2] * y.shape[3] * cin * k * k
    for t in range(_lib.CONV_TILES):
        if cfgs is not None and t not in cfgs and t != 5:
            continue
        d.tile = t + 1
        if not Engine._plan_ok(d, e):
            continue
        plan = Engine.plan(d, e)
        y.fill_(float("nan"))
        launch = lambda: _lib.call("qnn_qconv2d_fwd", ctypes.c_void_p(xq_ptr), _lib.ptr(m._qpack.wq), ctypes.byref(d),
                                   ctypes.byref(e), st_)
        launch()
        torch.cuda.synchronize()
        out = y.clone()
        if ref is None and t == 5:
            ref = out
        times = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            times.append((e0, e1))
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in times)[len(times) // 2]
        rows.append({"layer": name, "cfg": t, "tile": [plan[1], plan[2]], "blocks": plan[3], "us": round(ms * 1e3, 2),
                     "tops": round(ops / ms / 1e9, 1), "frac": round(ops / ms / 1e9 / PEAK, 4), "out": out})
    d.tile = 0
    for r in rows:
        r["equal_cfg5"] = None if ref is None else bool(torch.equal(r.pop("out"), ref))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--json")
    ap.add_argument("--cfgs", nargs="*", type=int, help="only these configurations (and 5, the reference)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    _lib.load()
    out = open(a.json, "w") if a.json else None
    for name, shape in LAYERS.items():
        if a.only and not any(o in name for o in a.only):
            continue
        rows = sweep(name, shape, a.reps, dev, a.cfgs)
        best = min(rows, key=lambda r: r["us"])
        for r in rows:
            line = json.dumps(r)
            print(line + ("   <== best" if r is best else ""), flush=True)
            if out:
                out.write(line + "\n")
    if out:
        out.close()


if __name__ == "__main__":
    main()
