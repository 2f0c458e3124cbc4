#!/usr/bin/env python3
"""Compare every residual code chain of the engine with the module path's fp32 block
outputs (which block first diverges).  python tools/debug_chain.py [fixture] [batch]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "quantized.pytorch_amd"), os.path.join(HERE, "tests")]

import torch  # noqa: E402

from conftest import load_fixture  # noqa: E402
from fixtures_util import build_model  # noqa: E402
from qnn import synthetic  # noqa: E402
from qnn.engine import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "model_resnet18_imagenet"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
d = load_fixture(name)
model, x = build_model(d)
dev = torch.device("cuda:0")
model = model.to(dev).eval()
x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 91).to(dev)
outs = []
mods = [model.maxpool if isinstance(model.maxpool, torch.nn.MaxPool2d) else model.relu]
mods += Engine._blocks(model)
hooks = [m.register_forward_hook(lambda m, i, o: outs.append(o.detach().clone())) for m in mods]
with torch.no_grad():
    model(x)
for h in hooks:
    h.remove()
eng = Engine(model, batch=batch, graph=False, autotune=False)
eng(x)
torch.cuda.synchronize()
for k, act in enumerate(eng.block_acts):
    ref = outs[k].permute(0, 2, 3, 1).reshape(-1, act.C)
    tag = f"act {k} {act.H}x{act.W}x{act.C}"
    if act.res is None:
        print(tag, "no residual representation")
        continue
    f32, links, relu0 = act.res
    r = eng.residual_value(act)
    bad = (r != ref).sum().item()
    print(tag, f"f32={'yes' if f32 is not None else 'no'} links={len(links)} relu0={relu0} "
          f"mismatches={bad}/{ref.numel()} maxdiff={(r - ref).abs().max().item():.3e}", flush=True)
