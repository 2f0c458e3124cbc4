#!/usr/bin/env python3
"""Phase breakdown of the stem max-pool kernel (stem_pool.hip) from its QNN_STAMP build.

    QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_spstamp.so python tools/sp_stamps.py --depth 18 --batch 128

Per wave: cycles in the prologue (epilogue data, tables, weights, first band), at the item tops
(band wait + barrier), in the stem tiles, at the mid barrier, in the pooling; items per block;
the block lifetimes (s_memrealtime, 100 MHz).  Stamps fence the phases: use the shares.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "quantized.pytorch_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth)
    eng = Engine(model, batch=a.batch, graph=False, autotune=False)
    eng.input.copy_(synthetic.input_batch(tuple(eng.input.shape), 1234).to(dev))
    st = _lib.stream_of(eng.input)
    lib = _lib.load()
    fn = lib.qnn_debug_stamps_sp
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    idx = eng.launch_names.index("qnn_qconv2d_maxpool_fwd")
    with torch.no_grad():
        eng()
        for _ in range(3):
            eng.ops[idx](st)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        eng.ops[idx](st)
        ev[1].record()
        torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3
    n = (1 << 16) // 64
    buf = np.zeros(n * 8 * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    w = buf.reshape(n, 8, 8).astype(np.float64)
    w = w[w[:, 0, 7] > 0]  # blocks that ran
    cyc = w[:, :, 2:7]
    tot = cyc.sum(-1)
    names = ["prologue", "item-tops", "tiles", "mid-barrier", "pooling"]
    m = cyc.mean((0, 1))
    life = (w[:, :, 1].max(1) - w[:, :, 0].min(1)) / 100.0
    print(f"stem max-pool resnet{a.depth} b{a.batch}: {us:.1f} us (stamped), {len(w)} blocks, items/block mean "
          f"{w[:, 0, 7].mean():.2f} max {w[:, 0, 7].max():.0f}; wave cycles mean {tot.mean():.0f}: " +
          "  ".join(f"{nm}={v:.0f} ({100 * v / tot.mean():.1f}%)" for nm, v in zip(names, m)) +
          f"; per item: tiles {m[2] / w[:, 0, 7].mean():.0f}, pooling {m[4] / w[:, 0, 7].mean():.0f} cycles; "
          f"block life mean {life.mean():.2f} max {life.max():.2f} us", flush=True)
    # spread of the per-wave tile phase (the waves of a block wait for the slowest at the mid barrier)
    tw = w[:, :, 4] / np.maximum(w[:, :, 7], 1)
    print(f"   tiles per item per wave: min {tw.min():.0f} mean {tw.mean():.0f} max {tw.max():.0f}; "
          f"pooling per item per wave: min {(w[:, :, 6] / w[:, :, 7]).min():.0f} max {(w[:, :, 6] / w[:, :, 7]).max():.0f}")


if __name__ == "__main__":
    main()
