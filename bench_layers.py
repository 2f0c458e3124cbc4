#!/usr/bin/env python3
"""Per-layer timing of the int8 MFMA conv kernel on the SURVEY.md §8(d) shapes.

For each layer: the QConv2d module path (quantize NCHW->NHWC8 + MFMA conv, fp32
NCHW out) and the conv kernel alone, HIP-event timed on the launch stream,
reported as int8 TOP/s against the 5 POPS dense peak and as algorithmic GB/s.

    python bench_layers.py [--reps 20] [--only headline]
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
import torch.nn as nn  # noqa: E402

from qnn import _lib, synthetic  # noqa: E402
from qnn.quantize import QConv2d  # noqa: E402

PEAK = 5000.0
# name: (cin, cout, k, stride, pad, N, H)
LAYERS = {
    "headline_r50_l3_3x3_256": (256, 256, 3, 1, 1, 256, 14),
    "r50_l4_3x3_512": (512, 512, 3, 1, 1, 256, 7),
    "r50_l1_3x3_64": (64, 64, 3, 1, 1, 256, 56),
    "r18_l1_3x3_64": (64, 64, 3, 1, 1, 128, 56),
    "r18_l2_3x3_128": (128, 128, 3, 1, 1, 128, 28),
    "r18_l3_3x3_256": (256, 256, 3, 1, 1, 128, 14),
    "r18_l4_3x3_512": (512, 512, 3, 1, 1, 128, 7),
    "r18_stem_7x7": (3, 64, 7, 2, 3, 128, 224),
    "r50_1x1_1024_256": (1024, 256, 1, 1, 0, 256, 14),
    "r50_1x1_256_1024": (256, 1024, 1, 1, 0, 256, 14),
}


def run(name, cfg, reps, dev, tile=None):
    cin, cout, k, st, pd, N, H = cfg
    m = QConv2d(cin, cout, k, stride=st, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
    if tile is not None:
        m.qnn_tile = tile + 1  # force tile configuration `tile` (qnn_conv_desc.tile)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 1)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(3.0)
    wrap = wrap.to(dev).eval()
    x = (torch.randn(N, cin, H, H, device=dev).relu_())
    with torch.no_grad():
        for _ in range(3):
            wrap(x)
        torch.cuda.synchronize()
        timer = _lib.LaunchTimer(["qnn_qconv2d_fwd", "qnn_quantize_nchw_to_nhwc8", "qnn_quantize_nchw_to_s2d8"])
        _lib.set_timer(timer)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            y = wrap(x)
        e1.record()
        _lib.set_timer(None)
        torch.cuda.synchronize()
    d = timer.durations_ms()
    cfg, bm, bn, nb = (ctypes.c_int() for _ in range(4))
    _lib.call("qnn_conv_plan", *(ctypes.byref(v) for v in m._last_conv), ctypes.byref(cfg), ctypes.byref(bm),
              ctypes.byref(bn), ctypes.byref(nb))
    conv = [ms for n, ms in d if n == "qnn_qconv2d_fwd"]
    quant = [ms for n, ms in d if n != "qnn_qconv2d_fwd"]
    conv_ms = sum(conv) / len(conv)
    mod_ms = e0.elapsed_time(e1) / reps
    Ho = y.shape[2]
    ops = 2 * N * cout * Ho * Ho * cin * k * k
    bytes_conv = N * H * H * ((cin + 15) // 16 * 16) + cout * k * k * cin + 4 * N * cout * Ho * Ho
    return {"layer": name, "gemm_MxNxK": [N * Ho * Ho, cout, cin * k * k], "gop": round(ops / 1e9, 2),
            "cfg": cfg.value, "tile": [bm.value, bn.value], "blocks": nb.value,
            "conv_us": round(conv_ms * 1e3, 2), "conv_tops": round(ops / conv_ms / 1e9, 1),
            "conv_frac": round(ops / conv_ms / 1e9 / PEAK, 4), "conv_alg_GBs": round(bytes_conv / conv_ms / 1e6, 1),
            "quantize_us": round(sum(quant) / len(quant) * 1e3, 2), "module_us": round(mod_ms * 1e3, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--tiles", nargs="*", type=int, help="force each of these tile configurations in turn")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    _lib.load()
    for name, cfg in LAYERS.items():
        if a.only and not any(o in name for o in a.only):
            continue
        for t in (a.tiles or [None]):
            print(json.dumps(run(name, cfg, a.reps, dev, t)), flush=True)


if __name__ == "__main__":
    main()
