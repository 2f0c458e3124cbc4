"""Split-K configurations (ids 44-45: configuration 11's tile with the K stages in 2 / 4 slices,
int32 partials in the caller's workspace, the last slice of a tile adds the others' and runs the
epilogue; include/qnn.h qnn_conv_desc.ksplit_*).

Integer partial sums are exact in any order, so every output must be bitwise the unsplit one's:
the engine at the ResNet-18 bench batch with each split configuration forced on every contraction
it is built for, twice (the per-tile counters are left at zero for the next launch and the
arrival order differs run to run), against the module path; and without a workspace (the
drop-in module path) the configurations are refused, never substituted.
"""
import functools

import pytest
import torch

from conftest import load_fixture
from fixtures_util import build_model
from qnn import _lib, synthetic

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=None)
def _model(fixture, batch):
    d = load_fixture(fixture)
    model, _ = build_model(d)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 91)
    return model, x


def _feat(model, x):
    feats = {}
    pool = model.avg_pool if hasattr(model, "avg_pool") else model.avgpool
    h = pool.register_forward_hook(lambda m, i, o: feats.__setitem__("x", i[0].detach().clone()))
    with torch.no_grad():
        model(x)
    h.remove()
    return feats["x"].permute(0, 2, 3, 1)


@pytest.mark.parametrize("fixture,batch", [("model_resnet18_imagenet", 128), ("model_resnet50_imagenet", 16)])
def test_ksplit_engine_bitwise(gpu, fixture, batch):
    from qnn.engine import Engine
    model, x = _model(fixture, batch)
    model = model.to(gpu)
    xg = x.to(gpu)
    ref = _feat(model, xg)
    for t in (44, 45):
        eng = Engine(model, batch=batch, graph=False, tile=t)
        forced = [n for n, (_i, d, _e) in enumerate(eng.convs) if d.tile == t + 1]
        assert len(forced) >= 4, f"configuration {t} is built for too few contractions: {forced}"
        for rep in range(2):
            eng(xg)
            torch.cuda.synchronize()
            assert torch.equal(eng.head_input, ref), f"configuration {t} run {rep}: engine != module path"
        print(f"{fixture} b{batch}: split-K configuration {t} on contractions {forced}")


def test_ksplit_refused_without_workspace(gpu):
    from qnn.engine import Engine
    model, x = _model("model_resnet18_imagenet", 8)
    model = model.to(gpu)
    eng = Engine(model, batch=8, graph=False, autotune=False)
    eng(x.to(gpu))
    st = _lib.stream_of(eng.input)
    n = 0
    for idx, d, e in eng.convs:
        d.ksplit_ws = None
        for t in (44, 45):
            d.tile = t + 1
            assert not Engine._plan_ok(d, e)
            with pytest.raises(_lib.QnnError, match="not built"):
                eng.ops[idx](st)
            n += 1
        d.tile = 0
    torch.cuda.synchronize()
    assert n > 0
