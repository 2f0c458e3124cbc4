#!/usr/bin/env python3
"""The drop-in module path (model(x), the reference's own forward: QConv2d / RangeBN / ReLU
modules, resnet_quantized.py) for rocprofv3 kernel statistics: 2 warm-up + N forwards.

    rocprofv3 --kernel-trace --stats -d out -- python3 tools/module_prof.py --depth 18 --batch 128
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "quantized.pytorch_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--fwd", type=int, default=5)
    a = ap.parse_args()
    import time
    import torch
    import bench
    from qnn import synthetic
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth)
    x = synthetic.input_batch((a.batch, 3, 224, 224), 1234).to(dev)
    with torch.no_grad():
        for _ in range(2):
            model(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.fwd):
            model(x)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.fwd
    print(f"module path resnet{a.depth} b{a.batch}: {dt * 1e3:.3f} ms per forward, {a.batch / dt:.1f} images/s")


if __name__ == "__main__":
    main()
