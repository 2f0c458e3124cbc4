#!/usr/bin/env python3
"""Per-launch profile of the fused engine: every kernel of one ResNet forward,
HIP-event timed on its launch stream, with the conv's GEMM shape, int8 TOP/s and
algorithmic GB/s (codes in + weights + codes/fp32 out).

    python profile_engine.py [--depth 18] [--batch 128] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "quantized.pytorch_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tile", type=int, default=None, help="force this tile configuration where it is built")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    _lib.load()
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch, graph=False, tile=a.tile)
    eng.input.copy_(synthetic.input_batch((a.batch, 3, 224, 224), 1234).to(dev))
    descs = [k for k in eng.keep if isinstance(k, _lib.ConvDesc)]
    epis = [k for k in eng.keep if isinstance(k, _lib.Epilogue)]
    timer = _lib.LaunchTimer(set(eng.launch_names))
    with torch.no_grad():
        eng()
        _lib.set_timer(timer)
        for _ in range(a.reps):
            eng()
        _lib.set_timer(None)
    d = timer.durations_ms()
    n = len(eng.ops)
    rows = []
    ci = 0
    for i in range(n):
        name = d[i][0]
        ms = sum(d[r * n + i][1] for r in range(a.reps)) / a.reps
        row = {"i": i, "kernel": name, "us": round(ms * 1e3, 2)}
        if name == "qnn_qconv2d_fwd":
            c = descs[ci]
            cfg, bm, bn, nb = (ctypes.c_int() for _ in range(4))
            _lib.call("qnn_conv_plan", ctypes.byref(c), ctypes.byref(epis[ci]), ctypes.byref(cfg), ctypes.byref(bm),
                      ctypes.byref(bn), ctypes.byref(nb))
            ci += 1
            M = c.n * c.ho * c.wo
            K = c.kh * c.kw * c.cp
            ops = 2 * M * c.cout * K
            e = epis[ci - 1]
            # algorithmic bytes: the padded input codes + packed weights + every output written
            # (fp32 4 B/elem, codes 1 B/elem per consumer, RangeBN codes 1 B; + fp32 residual read)
            out_b = M * c.cout * ((4 if e.out_f32 else 0) + (1 if e.out_code0 else 0) + (1 if e.out_code1 else 0)
                                 + (1 if e.out_bncode else 0) + (4 if e.residual else 0))
            alg = c.n * c.hp * c.wp * c.cp + c.cout * c.kpad + out_b
            row.update(MxNxK=[M, c.cout, K], alg_bytes=alg, cfg=cfg.value, tile=[bm.value, bn.value], blocks=nb.value, tops=round(ops / ms / 1e9, 1), frac=round(ops / ms / 1e9 / 5000, 4))
        rows.append(row)
        print(json.dumps(row), flush=True)
    tot = sum(r["us"] for r in rows)
    conv = sum(r["us"] for r in rows if r["kernel"] == "qnn_qconv2d_fwd")
    print(json.dumps({"total_us": round(tot, 1), "conv_us": round(conv, 1), "launches": n}))


if __name__ == "__main__":
    main()
