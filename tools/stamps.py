#!/usr/bin/env python3
"""Phase breakdown of the conv kernel from the QNN_STAMP diagnostic build.

    QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_stamp.so python tools/stamps.py --layer headline
    QNN_LIB=... python tools/stamps.py --engine 4 15        (engine launch indices, ResNet-18 b128)

Per launch: mean per-wave cycles in prologue / issue / wait+barrier / compute / trailing
barrier / epilogue (shares only: stamps fence overlaps, never quote the build's time),
and the block timeline (s_memrealtime, 100 MHz): waves of residency, tail.
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

from qnn import _lib  # noqa: E402

NF = 10


def plan(d, e=None):
    """(cfg, waves per block, blocks) of the conv launch for descriptor d."""
    cfg, bm, bn, nblk = (ctypes.c_int() for _ in range(4))
    e = e if e is not None else _lib.Epilogue(mode=1)
    _lib.call("qnn_conv_plan", ctypes.byref(d), ctypes.byref(e), ctypes.byref(cfg), ctypes.byref(bm),
              ctypes.byref(bn), ctypes.byref(nblk))
    # qconv.hip CFG[].waves (0-17) and XCFG[].waves (50-55); other families are not stamped here
    waves = {**dict(enumerate([8, 8, 8, 4, 4, 2, 8, 8, 8, 8, 4, 4, 8, 8, 8, 4, 4, 2])),
             **dict(zip(range(50, 56), [4, 2, 4, 2, 8, 8]))}.get(cfg.value)
    return cfg.value, waves, nblk.value


def read(nblk, W):
    lib = _lib.load()
    fn, fe = lib.qnn_debug_stamps, lib.qnn_debug_epi
    fn.argtypes = fe.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    nblk = min(nblk, (1 << 20) // (10 * W), (1 << 18) // (4 * W))
    buf = np.zeros(nblk * W * NF, dtype=np.uint64)
    ebuf = np.zeros(nblk * W * 4, dtype=np.uint64)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    assert fe(ebuf.ctypes.data, ebuf.nbytes) == 0
    return buf.reshape(nblk, W, NF), ebuf.reshape(nblk, W, 4)


def report(tag, sts):
    st, ep = sts
    nblk = st.shape[0]
    w = st.astype(np.float64)
    cyc = w[:, :, 2:8]
    tot = cyc.sum(-1)
    names = ["prologue", "issue", "wait+bar", "compute", "-", "epilogue"]
    mean = cyc.mean((0, 1))
    print(f"== {tag}: blocks={nblk} stages={int(w[0, 0, 9])} wave-cycles mean={tot.mean():.0f} "
          f"(min {tot.min():.0f} max {tot.max():.0f})")
    print("   " + "  ".join(f"{n}={m:.0f} ({100 * m / mean.sum():.1f}%)" for n, m in zip(names, mean)))
    per_stage = mean[1:5].sum() / max(1, w[0, 0, 9])
    print(f"   per stage: {per_stage:.0f} cycles (issue {mean[1] / w[0, 0, 9]:.0f}, wait {mean[2] / w[0, 0, 9]:.0f}, "
          f"compute {mean[3] / w[0, 0, 9]:.0f}, bar2 {mean[4] / w[0, 0, 9]:.0f})")
    rs = w[:, 0, 0] - w[:, 0, 0].min()
    re_ = w[:, 0, 1] - w[:, 0, 0].min()
    life = (re_ - rs)
    print(f"   timeline (us): last end {re_.max() / 100:.1f}, block life mean {life.mean() / 100:.2f} "
          f"max {life.max() / 100:.2f}; starts: " +
          " ".join(f"{np.percentile(rs, q) / 100:.1f}" for q in (0, 25, 50, 75, 90, 100)))
    # residency: how many blocks alive at each time point
    ts = np.linspace(0, re_.max(), 12)
    alive = [int(((rs <= t) & (re_ > t)).sum()) for t in ts]
    print("   alive blocks over time: " + " ".join(map(str, alive)))
    em = ep.astype(np.float64).mean((0, 1))
    print(f"   epilogue split: staging+sync {em[0]:.0f}  pixel state {em[1]:.0f}  body {em[2]:.0f}")
    cu = (w[:, 0, 8].astype(np.int64))
    print(f"   distinct HW_IDs: {len(np.unique(cu))}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", nargs="*", default=[])
    ap.add_argument("--engine", nargs="*", type=int, default=[])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.layer:
        import bench_layers
        import torch.nn as nn
        from qnn import synthetic
        from qnn.quantize import QConv2d
        for name, cfg in bench_layers.LAYERS.items():
            if not any(o in name for o in a.layer):
                continue
            cin, cout, k, stv, pd, N, H = cfg
            m = QConv2d(cin, cout, k, stride=stv, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
            wrap = nn.Sequential(m)
            synthetic.init_params(wrap, 1)
            m.quantize_input.running_min.fill_(0.0)
            m.quantize_input.running_max.fill_(3.0)
            wrap = wrap.to(dev).eval()
            x = torch.randn(N, cin, H, H, device=dev).relu_()
            with torch.no_grad():
                for _ in range(3):
                    wrap(x)
            cfg_, W, nblk = plan(*m._last_conv)
            report(f"{name} cfg={cfg_}", read(nblk, W))
    if a.engine:
        import bench
        from qnn import synthetic
        from qnn.engine import Engine
        model = bench.build(dev, 18)
        eng = Engine(model, batch=128, graph=False)
        eng.input.copy_(synthetic.input_batch((128, 3, 224, 224), 1234).to(dev))
        descs = [k for k in eng.keep if isinstance(k, _lib.ConvDesc)]
        epis = [k for k in eng.keep if isinstance(k, _lib.Epilogue)]
        st = _lib.stream_of(eng.input)
        with torch.no_grad():
            eng()
            ci = 0
            for i, (name, op) in enumerate(zip(eng.launch_names, eng.ops)):
                op(st)
                if name != "qnn_qconv2d_fwd":
                    continue
                d, e = descs[ci], epis[ci]
                ci += 1
                if i not in a.engine:
                    continue
                M = d.n * d.ho * d.wo
                cfg_, W, nblk = plan(d, e)
                if W is None:
                    print(f"engine launch {i}: configuration {cfg_} is not a qconv.hip kernel (no stamps)")
                    continue
                report(f"engine launch {i} M={M} cout={d.cout} K={d.kh * d.kw * d.cp} cfg={cfg_}", read(nblk, W))


if __name__ == "__main__":
    main()
