#!/usr/bin/env python3
"""Where do two tile configurations disagree?  Drop-in QConv2d forward with cfg A vs cfg B
(default 5 vs the given one), mismatch count and the (n, c, h, w) extents of the mismatches.

    python tools/rb_debug.py --cfg 28 --shape 256 256 3 1 1 8 14
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "quantized.pytorch_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from qnn import _lib, synthetic  # noqa: E402
from qnn.quantize import QConv2d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, required=True)
    ap.add_argument("--ref", type=int, default=5)
    ap.add_argument("--shape", type=int, nargs=7, default=[256, 256, 3, 1, 1, 8, 14])
    a = ap.parse_args()
    cin, cout, k, st, pd, N, H = a.shape
    dev = torch.device("cuda:0")
    _lib.load()
    m = QConv2d(cin, cout, k, stride=st, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 1)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(3.0)
    wrap = wrap.to(dev).eval()
    x = torch.randn(N, cin, H, H, device=dev).relu_()
    outs = []
    for t in (a.ref, a.cfg):
        m.qnn_tile = t + 1
        with torch.no_grad():
            outs.append(wrap(x).clone())
    m.qnn_tile = 0
    torch.cuda.synchronize()
    diff = (outs[0] != outs[1])
    nbad = int(diff.sum())
    print(f"shape {a.shape} cfg {a.cfg} vs {a.ref}: {nbad} of {diff.numel()} differ, "
          f"max|d| {float((outs[0] - outs[1]).abs().max()):.3e}")
    if nbad:
        idx = diff.nonzero()
        for dim, name in enumerate("nchw"):
            v = idx[:, dim]
            print(f"  {name}: min {int(v.min())} max {int(v.max())} distinct {len(torch.unique(v))}")
        print("  first:", idx[:8].tolist())


if __name__ == "__main__":
    main()
