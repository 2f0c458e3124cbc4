"""Every tile configuration of the int8 contraction computes the same result.

qnn_qconv2d_fwd has several tile configurations (include/qnn.h, qnn_conv_plan); the
cost model and the engine's autotuner pick among them purely on speed, so each one
must be checked on its own (the reference's contraction: quantize.py:342-349):

* mode 0 (drop-in NCHW fp32) of every configuration against the oracle at the
  per-layer bar, on the shapes the benchmarks run: the headline ResNet-50 3x3
  256@14x14, the K=4608 512@7x7 3x3, the 64@56x56 3x3, 1x1 reduce / expand,
  the strided 1x1 downsample, the space-to-depth 7x7/2 stem and the classifier;
* mode 1 (fused chains) of every configuration bitwise against the module path
  (the engine with the configuration forced on every contraction it is built for);
* the engine at benchmark-scale batches (ResNet-18 b128, ResNet-50 b64) with its
  autotuned tiles, bitwise against the module path.
Configurations not built for an epilogue kind must be refused, not silently replaced.
"""
import functools

import pytest
import torch
import torch.nn as nn

from conftest import load_fixture
from fixtures_util import build_model
from oracle import qnn_oracle as O
from qnn import _lib, synthetic
from qnn.quantize import QConv2d, QLinear

pytestmark = pytest.mark.gpu

LAYER_TOL = 1e-5

# (name, cin, cout, k, stride, pad, N, H, W); k == 0: QLinear (H = W = 1)
SHAPES = [
    ("headline_3x3_256_14", 256, 256, 3, 1, 1, 8, 14, 14),
    ("k4608_3x3_512_7", 512, 512, 3, 1, 1, 8, 7, 7),
    ("r18_3x3_64_56", 64, 64, 3, 1, 1, 2, 56, 56),
    ("reduce_1x1_1024_256", 1024, 256, 1, 1, 0, 4, 14, 14),
    ("expand_1x1_64_256", 64, 256, 1, 1, 0, 2, 56, 56),
    ("ds_1x1_s2_256_512", 256, 512, 1, 2, 0, 4, 14, 14),
    ("stem_7x7_s2", 3, 64, 7, 2, 3, 2, 224, 224),
    ("fc_2048_1000", 2048, 1000, 0, 1, 0, 37, 1, 1),
    ("fc_512_1000_b128", 512, 1000, 0, 1, 0, 128, 1, 1),   # ResNet-18 head (configuration 44)
    ("fc_1024_1000_b37", 1024, 1000, 0, 1, 0, 37, 1, 1),   # MobileNet head, ragged batch
]


def _ntiles():
    return _lib.CONV_TILES


@functools.lru_cache(maxsize=None)
def _case(name):
    """(module on CPU, input, oracle output, range) for a shape (built once)."""
    _, cin, cout, k, st, pd, N, H, W = next(s for s in SHAPES if s[0] == name)
    rng = (0.0, 2.75)
    if k == 0:
        m = QLinear(cin, cout, num_bits_grad=8, biprecision=True)
        x = synthetic.input_batch((N, cin), 18, relu=True) * 0.6
    else:
        m = QConv2d(cin, cout, k, stride=st, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
        x = synthetic.input_batch((N, cin, H, W), 17, relu=True) * 1.1
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 3)
    m.quantize_input.running_min.fill_(rng[0])
    m.quantize_input.running_max.fill_(rng[1])
    wrap.eval()
    sd = {kk: v.clone() for kk, v in wrap.state_dict().items()}
    if k == 0:
        ref = O.qlinear(x, sd["0.weight"], sd["0.bias"], rng)
    else:
        ref = O.qconv2d(x, sd["0.weight"], sd.get("0.bias"), st, pd, 1, 1, rng)
    return wrap, x, ref


def _close(y, ref, tol=LAYER_TOL):
    y, ref = y.detach().float().cpu(), ref.detach().float().cpu()
    assert y.shape == ref.shape
    err = (y - ref).abs().max().item()
    bound = tol * ref.abs().max().item() + 1e-6
    assert err <= bound, f"max|dy|={err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("tile", range(_lib.CONV_TILES))
@pytest.mark.parametrize("name", [s[0] for s in SHAPES])
def test_every_tile_mode0_vs_oracle(gpu, name, tile):
    wrap, x, ref = _case(name)
    wrap = wrap.to(gpu)
    m = wrap[0]
    from qnn.engine import Engine
    with torch.no_grad():
        wrap(x.to(gpu))  # descriptors of this layer (cost-model tile)
    d, e = m._last_conv
    d.tile = tile + 1
    if not Engine._plan_ok(d, e):  # not built for / does not fit this layer: refused, never substituted
        m.qnn_tile = tile + 1
        try:
            with pytest.raises(_lib.QnnError, match="not built"):
                with torch.no_grad():
                    wrap(x.to(gpu))
        finally:
            m.qnn_tile = 0
        return
    m.qnn_tile = tile + 1
    try:
        with torch.no_grad():
            y = wrap(x.to(gpu))
        d, e = m._last_conv
        assert Engine.plan(d, e)[0] == tile, "the forced configuration was not the one launched"
    finally:
        m.qnn_tile = 0
    _close(y, ref)


def _module_feat(model, x):
    feats = {}
    pool = model.avg_pool if hasattr(model, "avg_pool") else model.avgpool
    h = pool.register_forward_hook(lambda m, i, o: feats.__setitem__("x", i[0].detach().clone()))
    with torch.no_grad():
        logits = model(x)
    h.remove()
    return logits, feats["x"]


@functools.lru_cache(maxsize=None)
def _model(fixture, batch):
    d = load_fixture(fixture)
    model, _ = build_model(d)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 91)
    return model, x


@pytest.mark.parametrize("tile", range(_lib.CONV_TILES))
@pytest.mark.parametrize("fixture,batch", [("model_resnet18_imagenet", 8), ("model_resnet50_imagenet", 4),
                                           ("model_mobilenet", 4)])
def test_every_tile_fused_bitwise_vs_module_path(gpu, fixture, batch, tile):
    from qnn.engine import Engine
    model, x = _model(fixture, batch)
    model = model.to(gpu)
    xg = x.to(gpu)
    _, feat = _module_feat(model, xg)
    eng = Engine(model, batch=batch, graph=False, tile=tile)
    forced = sum(1 for (k, _), (_i, d, _e) in zip(eng.tiles, eng.convs) if d.tile == tile + 1)
    if forced == 0:
        pytest.skip(f"configuration {tile} is built for no contraction of {fixture}")
    eng(xg)
    assert torch.equal(eng.head_input, feat.permute(0, 2, 3, 1)), f"tile {tile}: engine != module path"


def test_unbuilt_tile_is_refused(gpu):
    """A configuration not built for the epilogue kind is an argument error, never a silent
    substitute (the autotuner must not time one configuration under another's label)."""
    from qnn.engine import Engine
    model, x = _model("model_resnet50_imagenet", 4)
    model = model.to(gpu)
    eng = Engine(model, batch=4, graph=False, autotune=False)
    eng()  # every buffer holds real data
    st = _lib.stream_of(eng.input)
    for idx, d, e in eng.convs:
        for k in range(_lib.CONV_TILES):
            d.tile = k + 1
            if not Engine._plan_ok(d, e):
                with pytest.raises(_lib.QnnError, match="not built"):
                    eng.ops[idx](st)
        d.tile = 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("fixture,batch", [("model_resnet18_imagenet", 128), ("model_resnet50_imagenet", 64)])
def test_engine_bench_batch_bitwise_vs_module_path(gpu, fixture, batch):
    """The engine at a benchmark-scale batch, autotuned, against the module path: the
    kernels behind the headline img/s are the ones checked."""
    from qnn.engine import Engine
    model, x = _model(fixture, batch)
    model = model.to(gpu)
    xg = x.to(gpu)
    _, feat = _module_feat(model, xg)
    eng = Engine(model, batch=batch)
    eng(xg)
    print(f"{fixture} b{batch} autotuned tiles: {[k for k, _ in eng.tiles]}")
    assert torch.equal(eng.head_input, feat.permute(0, 2, 3, 1))


@pytest.mark.parametrize("name", ["headline_3x3_256_14", "r18_3x3_64_56"])
def test_module_autotune_bitwise(gpu, name):
    """The drop-in module path's per-shape autotune picks a configuration built for the layer,
    remembers it per input shape, and changes nothing but speed: bitwise the cost model's
    output."""
    from qnn import quantize as Q
    wrap, x, ref = _case(name)
    wrap = wrap.to(gpu)
    m = wrap[0]
    xg = x.to(gpu)
    with torch.no_grad():
        y0 = wrap(xg)
    Q.MODULE_AUTOTUNE[0] = True
    try:
        with torch.no_grad():
            y1 = wrap(xg)
            y2 = wrap(xg)
    finally:
        Q.MODULE_AUTOTUNE[0] = False
    assert len(m._tuned) == 1
    k = next(iter(m._tuned.values()))
    assert 1 <= k <= _lib.CONV_TILES
    from qnn.engine import Engine
    assert Engine.plan(*m._last_conv)[0] == k - 1
    assert torch.equal(y0, y1) and torch.equal(y1, y2)
    _close(y1, ref)
