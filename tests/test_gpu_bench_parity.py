"""Parity at the benchmark batches and at natural occupancy.

* Resident-band configurations (qnn_conv_tile_kernel == "qconv_rb_kernel") at natural
  occupancy -- as many blocks per CU as registers and LDS allow, no LDS inflation -- on the
  ResNet-50 b256 shapes (the headline 256@14x14 3x3, the K=4608 512@7x7, the 128@28x28
  layer-2 3x3) and the 64-channel 56x56 band: bitwise against the ring kernel (config 5) and
  against the oracle at the per-layer bar; on the headline shape at least one configuration
  must really run two or more blocks per CU (qnn_conv_occupancy).  This is the test that
  reproduced the co-residency corruption (a weight load refilling an A operand right after
  the MFMA that reads it).
* Direct-fragment configurations where every persistent block loops over at least
  two pixel tiles (the loop and its next-tile prefetch, qconv_direct.hip), against the oracle.
* The engine at the bench batches of configs C3 (ResNet-50 b256) and C4 (MobileNet b512),
  autotuned, bitwise against the module path (resnet_quantized.py:93-113,
  mobilenet_quantized.py:33-53; the contraction is quantize.py:342-349).
"""
import ctypes
import functools

import pytest
import torch
import torch.nn as nn

from conftest import load_fixture
from fixtures_util import build_model
from oracle import qnn_oracle as O
from qnn import _lib, synthetic
from qnn.quantize import QConv2d

pytestmark = pytest.mark.gpu

LAYER_TOL = 1e-5
RING = 5


def _rb_ids():
    return _lib.tile_ids("qconv_rb_kernel")


def _direct_ids():
    return _lib.tile_ids("qconv_direct_kernel")


def _occupancy(d, e):
    cfg, bpc, lds, grid = (ctypes.c_int() for _ in range(4))
    _lib.call("qnn_conv_occupancy", ctypes.byref(d), ctypes.byref(e), ctypes.byref(cfg), ctypes.byref(bpc),
              ctypes.byref(lds), ctypes.byref(grid))
    return cfg.value, bpc.value, lds.value, grid.value


def _plan(d, e):
    from qnn.engine import Engine
    return Engine.plan(d, e)


@functools.lru_cache(maxsize=None)
def _layer(cin, cout, k, st, pd, N, H, seed):
    m = QConv2d(cin, cout, k, stride=st, padding=pd, bias=False, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, seed)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(2.75)
    wrap.eval()
    x = synthetic.input_batch((N, cin, H, H), seed + 1, relu=True) * 1.1
    return wrap, x


def _run(wrap, xg, tile):
    m = wrap[0]
    m.qnn_tile = tile + 1
    try:
        with torch.no_grad():
            y = wrap(xg)
        d, e = m._last_conv
        return y, d, e
    finally:
        m.qnn_tile = 0


def _oracle_rows(wrap, x, idx):
    """Oracle output of the images `idx` (the eval forward is per-sample independent)."""
    sd = {k: v.clone() for k, v in wrap.state_dict().items()}
    m = wrap[0]
    return O.qconv2d(x[idx], sd["0.weight"], sd.get("0.bias"), m.stride, m.padding, 1, 1, (0.0, 2.75))


def _close(y, ref, tol=LAYER_TOL):
    y, ref = y.detach().float().cpu(), ref.detach().float().cpu()
    err = (y - ref).abs().max().item()
    bound = tol * ref.abs().max().item() + 1e-6
    assert err <= bound, f"max|dy|={err:.3e} > {bound:.3e}"


RB_SHAPES = [  # (name, cin, cout, k, stride, pad, N, H)
    ("headline_3x3_256_14_b256", 256, 256, 3, 1, 1, 256, 14),
    ("k4608_3x3_512_7_b256", 512, 512, 3, 1, 1, 256, 7),
    ("l2_3x3_128_28_b256", 128, 128, 3, 1, 1, 256, 28),
    ("l1_3x3_64_56_b32", 64, 64, 3, 1, 1, 32, 56),
]


@pytest.mark.parametrize("name", [s[0] for s in RB_SHAPES])
def test_resident_band_natural_occupancy(gpu, name):
    _, cin, cout, k, st, pd, N, H = next(s for s in RB_SHAPES if s[0] == name)
    wrap, x = _layer(cin, cout, k, st, pd, N, H, 41)
    wrap = wrap.to(gpu)
    xg = x.to(gpu)
    y_ring, d, e = _run(wrap, xg, RING)
    idx = torch.tensor([0, 1, N - 2, N - 1])
    _close(y_ring[idx], _oracle_rows(wrap.cpu(), x, idx))
    wrap = wrap.to(gpu)
    ran = []
    for t in _rb_ids():
        d.tile = t + 1
        from qnn.engine import Engine
        if not Engine._plan_ok(d, e):
            continue
        cfg, bpc, lds, grid = _occupancy(d, e)
        assert cfg == t and 1 <= bpc and lds <= 160 * 1024
        y, _, _ = _run(wrap, xg, t)
        torch.cuda.synchronize()
        ndiff = int((y != y_ring).sum())
        assert ndiff == 0, f"config {t} ({bpc} blocks/CU, {lds} B LDS, grid {grid}): {ndiff} outputs != config {RING}"
        ran.append((t, bpc, grid))
    print(f"{name}: resident-band configurations (id, blocks/CU, grid) = {ran}")
    assert ran, "no resident-band configuration is built for this shape"
    if name.startswith("headline"):
        two = [r for r in ran if r[1] >= 2 and r[2] >= 2 * 256]
        assert two, f"no resident-band configuration runs two co-resident blocks per CU on a full grid: {ran}"


RBP_SHAPES = [  # (name, cin, cout, k, stride, pad, N, H): the two-team kernel's target layers
    ("headline_3x3_256_14_b256", 256, 256, 3, 1, 1, 256, 14),
    ("k4608_3x3_512_7_b256", 512, 512, 3, 1, 1, 256, 7),
    ("r18_3x3_256_14_b128", 256, 256, 3, 1, 1, 128, 14),
    ("ragged_3x3_256_14_b37", 256, 256, 3, 1, 1, 37, 14),
]


@pytest.mark.parametrize("name", [s[0] for s in RBP_SHAPES])
def test_two_team_resident_band_bench(gpu, name):
    """qconv_rbp_kernel (two priority teams, chunked band, LDS counters instead of barriers) on
    full grids: bitwise against the ring kernel, twice (run-to-run identical), and the ring
    kernel against the oracle on the first and last images."""
    _, cin, cout, k, st, pd, N, H = next(s for s in RBP_SHAPES if s[0] == name)
    wrap, x = _layer(cin, cout, k, st, pd, N, H, 43)
    wrap = wrap.to(gpu)
    xg = x.to(gpu)
    y_ring, d, e = _run(wrap, xg, RING)
    idx = torch.tensor([0, N - 1])
    _close(y_ring[idx], _oracle_rows(wrap.cpu(), x, idx))
    wrap = wrap.to(gpu)
    from qnn.engine import Engine
    ran = []
    for t in _lib.tile_ids("qconv_rbp_kernel"):
        d.tile = t + 1
        if not Engine._plan_ok(d, e):
            continue
        for rep in range(2):
            y, _, _ = _run(wrap, xg, t)
            torch.cuda.synchronize()
            ndiff = int((y != y_ring).sum())
            assert ndiff == 0, f"config {t} run {rep}: {ndiff} outputs != config {RING}"
        ran.append((t, Engine.plan(d, e)[3]))
    print(f"{name}: two-team configurations (id, grid) = {ran}")
    assert ran, "no two-team configuration is built for this shape"


DIRECT_SHAPES = [  # (name, direct-fragment configuration index, cin, cout, k, stride, pad, N, H)
    ("mbn_stem_s2d_3x3_32_b256", 0, 3, 32, 3, 2, 1, 256, 224),
    ("r_stem_s2d_7x7_64_b128", 1, 3, 64, 7, 2, 3, 128, 224),
    ("pw_1x1_64_128_56_b256", 2, 64, 128, 1, 1, 0, 256, 56),
    # K = 576 (3x3 on 64 channels, weights resident in VGPRs): ResNet layer 1 and the
    # stride-2 entry of layer 2, at the ResNet-18 bench batch
    ("r18_3x3_64_56_b128", 3, 64, 64, 3, 1, 1, 128, 56),
    ("r18_3x3_64_56_b128_noprefetch", 4, 64, 64, 3, 1, 1, 128, 56),
    ("r18_3x3_s2_64_128_b128", 3, 64, 128, 3, 2, 1, 128, 56),
]


@pytest.mark.parametrize("name", [s[0] for s in DIRECT_SHAPES])
def test_direct_fragment_persistent_loop(gpu, name):
    _, di, cin, cout, k, st, pd, N, H = next(s for s in DIRECT_SHAPES if s[0] == name)
    tile = _direct_ids()[di]
    wrap, x = _layer(cin, cout, k, st, pd, N, H, 43)
    wrap = wrap.to(gpu)
    xg = x.to(gpu)
    y, d, e = _run(wrap, xg, tile)
    cfg, bpc, lds, grid = _occupancy(d, e)
    tiles = _plan(d, e)[3]
    assert cfg == tile
    assert tiles >= 2 * grid, f"{tiles} pixel tiles over a grid of {grid}: a block must loop over >= 2 tiles"
    print(f"{name}: config {tile}, {bpc} blocks/CU, grid {grid}, {tiles} tiles ({tiles / grid:.1f} per block)")
    idx = torch.tensor([0, N // 2, N - 1])
    _close(y[idx], _oracle_rows(wrap.cpu(), x, idx))
    # every tile of the loop, the prefetched ones included: bitwise against a
    # non-persistent kernel (the ring kernel, config 11)
    from qnn.engine import Engine
    d.tile = 12
    if Engine._plan_ok(d, e):
        wrap = wrap.to(gpu)
        y_ring, _, _ = _run(wrap, xg, 11)
        assert torch.equal(y, y_ring)


def _module_feat(model, x):
    feats = {}
    pool = model.avg_pool if hasattr(model, "avg_pool") else model.avgpool
    h = pool.register_forward_hook(lambda m, i, o: feats.__setitem__("x", i[0].detach().clone()))
    with torch.no_grad():
        logits = model(x)
    h.remove()
    return logits, feats["x"]


@pytest.mark.parametrize("fixture,batch", [("model_resnet50_imagenet", 256), ("model_mobilenet", 512)])
def test_engine_bench_batch_bitwise_c3_c4(gpu, fixture, batch):
    from qnn.engine import Engine
    d = load_fixture(fixture)
    model, _ = build_model(d)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 93)
    model = model.to(gpu)
    xg = x.to(gpu)
    logits, feat = _module_feat(model, xg)
    eng = Engine(model, batch=batch)
    out = eng(xg)
    torch.cuda.synchronize()
    tiles = [k for k, _ in eng.tiles]
    print(f"{fixture} b{batch} autotuned tiles: {tiles}")
    assert torch.equal(eng.head_input, feat.permute(0, 2, 3, 1)), "engine != module path at the bench batch"
    multi = []
    for (k, _), (_i, dd, ee) in zip(eng.tiles, eng.convs):
        if k in _direct_ids():
            _, _, _, grid = _occupancy(dd, ee)
            multi.append(_plan(dd, ee)[3] / grid)
    if fixture == "model_mobilenet":
        assert multi and max(multi) >= 2, f"no direct-fragment launch loops over >= 2 tiles per block: {multi}"
    # the logits too: the engine's avg-pool sums in torch's AvgPool2d order
    assert torch.equal(out, logits), (out - logits).abs().max().item()


@pytest.mark.parametrize("fixture,batch", [("model_resnet50_imagenet", 256), ("model_resnet18_imagenet", 128)])
def test_engine_split_chain_bench_batch_bitwise(gpu, fixture, batch):
    """The split residual-chain epilogue (qnn_chain_epilogue) at the bench batches (C2, C3):
    the launch walks many pixel tiles per block; head input and logits bitwise the module path."""
    from qnn.engine import Engine
    d = load_fixture(fixture)
    model, _ = build_model(d)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 94)
    model = model.to(gpu)
    xg = x.to(gpu)
    logits, feat = _module_feat(model, xg)
    eng = Engine(model, batch=batch, split_chain=True)
    out = eng(xg)
    assert "qnn_chain_epilogue" in eng.launch_names
    assert torch.equal(eng.head_input, feat.permute(0, 2, 3, 1)), "split-chain engine != module path"
    assert torch.equal(out, logits)
