#!/usr/bin/env python3
"""Time chosen launches of one engine forward (any kernel, by launch index) with HIP events
on the launch stream -- for A/B builds of a kernel (QNN_LIB=...).

    python tools/time_ops.py --depth 18 --batch 128 --ops 0 1 [--reps 20]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "quantized.pytorch_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--ops", nargs="*", type=int, default=[1])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    from qnn import _lib, synthetic
    from qnn.engine import Engine
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch, graph=False, autotune=False)
    eng.input.copy_(synthetic.input_batch(tuple(eng.input.shape), 1234).to(dev))
    st = _lib.stream_of(eng.input)
    with torch.no_grad():
        eng()
        torch.cuda.synchronize()
        for idx in a.ops:
            for _ in range(3):
                eng.ops[idx](st)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(a.reps):
                eng.ops[idx](st)
            ev[1].record()
            ev[1].synchronize()
            print(f"{os.path.basename(_lib.LIB_PATH)} launch {idx} {eng.launch_names[idx]}: "
                  f"{ev[0].elapsed_time(ev[1]) / a.reps * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
