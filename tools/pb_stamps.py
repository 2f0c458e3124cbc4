#!/usr/bin/env python3
"""Phase breakdown of the persistent-band kernel (qconv_pb.hip) from its QNN_STAMP build.

    QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_pbstamp.so python tools/pb_stamps.py --launch 3 4 --tiles 45 46 47

Per wave: cycles from kernel start to the first band (weights, epilogue data, band 0), in the
band tops (DMA wait + barrier + channel sums + barrier), in the tile contractions, in the
epilogues; tiles and bands per wave; the block timeline (s_memrealtime, 100 MHz).  Stamps fence
the phases: use the shares, not the absolute times.
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
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--launch", nargs="*", type=int, default=[3, 4])
    ap.add_argument("--tiles", nargs="*", type=int, default=[45, 46, 47])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model = bench.build(dev, a.depth, arch=a.model)
    eng = Engine(model, batch=a.batch, graph=False, autotune=False)
    eng.input.copy_(synthetic.input_batch(tuple(eng.input.shape), 1234).to(dev))
    st = _lib.stream_of(eng.input)
    lib = _lib.load()
    fn = lib.qnn_debug_stamps_pb
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    with torch.no_grad():
        eng()
        torch.cuda.synchronize()
        for idx, d, e in eng.convs:
            if idx not in a.launch:
                continue
            keep = d.tile
            for k in a.tiles:
                d.tile = k + 1
                if not Engine._plan_ok(d, e):
                    print(f"launch {idx} cfg {k}: not built")
                    continue
                for _ in range(3):
                    eng.ops[idx](st)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                eng.ops[idx](st)
                ev[1].record()
                torch.cuda.synchronize()
                us = ev[0].elapsed_time(ev[1]) * 1e3
                grid = ctypes.c_int()
                _lib.call("qnn_conv_occupancy", ctypes.byref(d), ctypes.byref(e), None, None, None, ctypes.byref(grid))
                n = min(grid.value, (1 << 19) // 64)
                buf = np.zeros(n * 4 * 16, dtype=np.uint64)
                assert fn(buf.ctypes.data, buf.nbytes) == 0
                w = buf.reshape(n, 4, 16).astype(np.float64)
                cyc = w[:, :, 2:6]
                life = (w[:, :, 1] - w[:, :, 0]).max(1) / 100.0  # us per block
                start = w[:, :, 0].min(1)
                tot = cyc.sum(-1)
                names = ["prologue", "band-tops", "contraction", "epilogue"]
                m = cyc.mean((0, 1))
                print(f"launch {idx} cp{d.cp}->{d.cout} cfg {k}: {us:.1f} us (stamped), grid {grid.value}, "
                      f"wave cycles mean {tot.mean():.0f} max {tot.max():.0f}: " +
                      "  ".join(f"{nm}={v:.0f} ({100 * v / tot.mean():.1f}%)" for nm, v in zip(names, m)) +
                      f"; tiles/wave mean {w[:, :, 6].mean():.2f} max {w[:, :, 6].max():.0f}, bands/block mean "
                      f"{w[:, 0, 7].mean():.2f} max {w[:, 0, 7].max():.0f}; per tile: contraction "
                      f"{(cyc[:, :, 2].sum() / w[:, :, 6].sum()):.0f}, epilogue {(cyc[:, :, 3].sum() / w[:, :, 6].sum()):.0f} cycles; "
                      f"block life mean {life.mean():.2f} max {life.max():.2f} us, starts spread "
                      f"{(start.max() - start.min()) / 100.0:.2f} us", flush=True)
                pro = w[:, :, 8:12].mean((0, 1))
                print("   prologue (cycles from start): epilogue data + classes issued {:.0f}, weights DMA issued {:.0f}, "
                      "all landed + barrier {:.0f}, weights in VGPRs + barrier {:.0f}".format(*pro), flush=True)
            d.tile = keep


if __name__ == "__main__":
    main()
