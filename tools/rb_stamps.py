#!/usr/bin/env python3
"""Phase breakdown of the resident-band conv kernels from their QNN_STAMP builds.

    QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_stamp_rb.so python tools/rb_stamps.py [--tiles 26 29]
    QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbpstamp.so python tools/rb_stamps.py --kernel rbp --tiles 40 41

For each ResNet layer picked (engine launch of the fused forward, its real epilogue kind) the
launch is forced onto each resident-band configuration and run; per wave: cycles until the
band landed (prologue), in the K loop, in the channel sums, in the epilogue; and the block
timeline (s_memrealtime, 100 MHz).  Stamps fence the phases: use the shares, not the times.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quantized.pytorch_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402


KERNEL = "rb"


def run(eng, idx, d, e, tile, reps):
    d.tile = tile + 1
    if not Engine._plan_ok(d, e):
        d.tile = 0
        return None
    cfg, bm, bn, nblk = (ctypes.c_int() for _ in range(4))
    _lib.call("qnn_conv_plan", ctypes.byref(d), ctypes.byref(e), ctypes.byref(cfg), ctypes.byref(bm),
              ctypes.byref(bn), ctypes.byref(nblk))
    st = _lib.stream_of(eng.input)
    for _ in range(reps):
        eng.ops[idx](st)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.ops[idx](st)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3
    lib = _lib.load()
    fn = getattr(lib, "qnn_debug_stamps_" + KERNEL)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    W = 8
    S = 16 if KERNEL == "rbp" else 8  # stamp slots per wave (rb, rs: 8)
    n = min(nblk.value, (1 << 18) // (S * W))
    buf = np.zeros(n * W * S, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    d.tile = 0
    return us, nblk.value, buf.reshape(n, W, S).astype(np.float64)


def report(tag, us, nblk, w):
    cyc = w[:, :, 2:8]
    mean = cyc.mean((0, 1))
    tot = cyc.sum(-1).mean()
    names = {"rb": ["band", "k-loop", "sums", "staging", "epi", "drain"],
             "rbp": ["chunk0", "k-loop", "sums", "epidata", "epi", "drain"],
             "rs": ["issue", "wait0", "barrier0", "k-loop", "epi", "drain"]}[KERNEL]
    print(f"== {tag}: {us:.1f} us (stamped build), blocks={nblk}, wave-cycles {tot:.0f}: " +
          "  ".join(f"{a}={m:.0f} ({100 * m / tot:.1f}%)" for a, m in zip(names, mean)))
    if KERNEL == "rs":  # the SIMD pairs: waves 0-3 (priority 1 in the PRIO configurations) vs 4-7
        for tm in (0, 1):
            c = cyc[:, 4 * tm:4 * tm + 4]
            cum = np.cumsum(c.mean((0, 1)))
            print(f"   waves {4 * tm}-{4 * tm + 3}: " + "  ".join(f"{a}={m:.0f}" for a, m in zip(names, c.mean((0, 1)))) +
                  "   cumulative: " + " ".join(f"{x:.0f}" for x in cum))
    if KERNEL == "rbp":  # the two teams (waves 0-3 at priority 2, 4-7 at 0)
        for tm in (0, 1):
            c = cyc[:, 4 * tm:4 * tm + 4]
            cum = np.cumsum(c.mean((0, 1)))
            print(f"   team {tm}: " + "  ".join(f"{a}={m:.0f}" for a, m in zip(names, c.mean((0, 1)))) +
                  "   cumulative end of each phase: " + " ".join(f"{x:.0f}" for x in cum))
        pro = w[:, :, 8:12].mean((0, 1))
        print("   prologue (cycles from start, all waves): barrier passed {:.0f}, chunk 0 + weights issued {:.0f}, "
              "own pieces landed {:.0f}, summed {:.0f}".format(*pro))
    rs = w[:, 0, 0] - w[:, 0, 0].min()
    re_ = w[:, 0, 1] - w[:, 0, 0].min()
    life = re_ - rs
    clk = tot / (life.mean() / 100) / 1e3 if life.mean() > 0 else 0
    print(f"   timeline (us): last end {re_.max() / 100:.1f}, block life mean {life.mean() / 100:.2f} "
          f"max {life.max() / 100:.2f} (clock ~{clk:.2f} GHz); starts p0/50/90/100: " +
          " ".join(f"{np.percentile(rs, q) / 100:.1f}" for q in (0, 50, 90, 100)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tiles", nargs="*", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kernel", choices=("rb", "rbp", "rs"), default="rb")
    ap.add_argument("--only3x3", default="")
    a = ap.parse_args()
    global KERNEL
    KERNEL = a.kernel
    dev = torch.device("cuda:0")
    _lib.load()
    model = bench.build(dev, a.depth)
    eng = Engine(model, batch=a.batch, graph=False, autotune=False)
    eng.input.copy_(synthetic.input_batch((a.batch, 3, 224, 224), 1234).to(dev))
    with torch.no_grad():
        eng()
    torch.cuda.synchronize()
    tiles = a.tiles or [26, 27, 28, 29]
    seen = set()
    for idx, d, e in eng.convs:
        if d.kh != 3:
            continue
        key = (d.cp, d.cout, d.ho, d.sh, e.lut, e.nres)
        if key in seen:
            continue
        seen.add(key)
        for t in tiles:
            r = run(eng, idx, d, e, t, a.reps)
            if r is None:
                continue
            report(f"launch {idx} cp{d.cp}->{d.cout} {d.ho}x{d.wo} s{d.sh} lut={e.lut is not None and bool(e.lut)} "
                   f"nres={e.nres} cfg {t}", *r)


if __name__ == "__main__":
    main()
