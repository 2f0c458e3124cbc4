#!/usr/bin/env python3
"""Time one engine contraction with parts of its fused epilogue switched off in the
descriptor (outputs become wrong; timing only): which part of EK_GEN costs what.
    python tools/epi_ablate.py [launch ...]      (ResNet-18 b128 engine launch indices)"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "quantized.pytorch_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from qnn import _lib, synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402

dev = torch.device("cuda:0")
model = bench.build(dev, 18)
eng = Engine(model, batch=128, graph=False)
eng.input.copy_(synthetic.input_batch((128, 3, 224, 224), 1234).to(dev))
eng()
st = _lib.stream_of(eng.input)
conv = {i: (d, e) for i, d, e in eng.convs}


def timeit(op, reps=20):
    op(st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        op(st)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for i in [int(v) for v in sys.argv[1:]] or [3, 4, 5, 6]:
    d, e = conv[i]
    saved = {f: getattr(e, f) for f, _ in _lib.Epilogue._fields_ if f != "res"}
    variants = [("as planned", {})]
    if e.nres:
        variants.append(("no chain", {"nres": 0, "res_relu0": 0}))
    if e.out_code1:
        variants.append(("no code1", {"out_code1": None}))
    if e.out_bncode:
        variants.append(("no bncode", {"out_bncode": None}))
    variants.append(("bn+relu+code0 only", {"nres": 0, "res_relu0": 0, "out_code1": None, "out_bncode": None}))
    print(f"launch {i}: cout={d.cout} K={d.kh * d.kw * d.cp} plan={Engine.plan(d, e)} lut={bool(e.lut)} "
          f"nres={e.nres} code1={bool(e.out_code1)} bncode={bool(e.out_bncode)}", flush=True)
    for name, ch in variants:
        for f, v in ch.items():
            setattr(e, f, v)
        print(f"   {name:22s} {timeit(eng.ops[i]):8.2f} us", flush=True)
        for f, v in saved.items():
            setattr(e, f, v)
eng()  # restore every buffer
torch.cuda.synchronize()
