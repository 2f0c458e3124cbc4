#!/usr/bin/env python3
"""Time chosen engine contraction launches under each tile configuration (HIP events on
the launch stream), reporting the configurations that refuse the layer and why.

    python tools/time_launch.py --model mobilenet --batch 512 --launch 1 3 --tiles 15 30 31
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quantized.pytorch_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--launch", nargs="*", type=int, default=[1])
    ap.add_argument("--tiles", nargs="*", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch, graph=False, autotune=False)
    eng.input.copy_(synthetic.input_batch(tuple(eng.input.shape), 1234).to(dev))
    st = _lib.stream_of(eng.input)
    with torch.no_grad():
        eng()
        torch.cuda.synchronize()
        for idx, d, e in eng.convs:
            if idx not in a.launch:
                continue
            keep = d.tile
            for k in (a.tiles if a.tiles is not None else range(_lib.CONV_TILES)):
                d.tile = k + 1
                try:
                    eng.ops[idx](st)
                except _lib.QnnError as err:
                    print(f"launch {idx} cfg {k}: refused ({err})")
                    continue
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(a.reps):
                    eng.ops[idx](st)
                ev[1].record()
                ev[1].synchronize()
                print(f"launch {idx} cp{d.cp}->{d.cout} k{d.kh}x{d.kw} kpad{d.kpad} M={d.n * d.ho * d.wo} "
                      f"cfg {k}: {ev[0].elapsed_time(ev[1]) / a.reps * 1e3:.1f} us", flush=True)
            d.tile = keep


if __name__ == "__main__":
    main()
