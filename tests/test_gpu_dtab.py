"""Table-epilogue configurations (qnn_conv_tile_kernel == "qconv_dtab_kernel", ids 42-43).

They evaluate the general chain of the short-K 1x1 layers -- RangeBN, the residual (fp32
checkpoint and/or up to four code-chain links), ReLU, codes / RangeBN input codes out -- by
looking up per-channel tables of the RangeBN and chain-link functions of a code, evaluated once
per block with the same fp32 ops (csrc/qconv_direct.hip, namespace dt).  So every output must be
bitwise the module path's (quantize.py:461-499 op order), on:

* ResNet-50 at batch 32 (layer 1's expand convs: 100 352 pixels, chains of 1-3 links; layer 3:
  the 1024-channel expand with 64 channel tiles and the XCD-grouped block order) and a ragged
  batch 7 (pixel tiles past the batch), each configuration forced on every contraction it is
  built for, run twice (run-to-run identical);
* the mode-0 drop-in layer and the LUT / BN-code epilogue kinds are refused ("not built"),
  never substituted.
"""
import functools

import pytest
import torch

from conftest import load_fixture
from fixtures_util import build_model
from qnn import _lib, synthetic

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=None)
def _model(batch):
    d = load_fixture("model_resnet50_imagenet")
    model, _ = build_model(d)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 91)
    return model, x


def _module_feat(model, x):
    feats = {}
    pool = model.avg_pool if hasattr(model, "avg_pool") else model.avgpool
    h = pool.register_forward_hook(lambda m, i, o: feats.__setitem__("x", i[0].detach().clone()))
    with torch.no_grad():
        model(x)
    h.remove()
    return feats["x"]


@pytest.mark.parametrize("batch", [32, 7])
def test_dtab_engine_bitwise_vs_module_path(gpu, batch):
    from qnn.engine import Engine
    model, x = _model(batch)
    model = model.to(gpu)
    xg = x.to(gpu)
    feat = _module_feat(model, xg).permute(0, 2, 3, 1)
    ids = _lib.tile_ids("qconv_dtab_kernel")
    assert ids == [42, 43]
    for t in ids:
        eng = Engine(model, batch=batch, graph=False, tile=t)
        forced = [i for i, ((k, _), (_n, d, _e)) in enumerate(zip(eng.tiles, eng.convs)) if d.tile == t + 1]
        assert forced, f"configuration {t} is built for no contraction of ResNet-50"
        for rep in range(2):
            eng(xg)
            torch.cuda.synchronize()
            assert torch.equal(eng.head_input, feat), f"configuration {t} run {rep}: engine != module path"
        print(f"b{batch}: configuration {t} forced on contractions {forced}")


def test_dtab_refuses_other_epilogue_kinds(gpu):
    """Mode 0 (NCHW fp32) and the LUT epilogue of a plain conv are not built here."""
    from qnn.engine import Engine
    model, x = _model(7)
    model = model.to(gpu)
    eng = Engine(model, batch=7, graph=False, autotune=False)
    eng(x.to(gpu))
    st = _lib.stream_of(eng.input)
    refused = built = 0
    for idx, d, e in eng.convs:
        for t in _lib.tile_ids("qconv_dtab_kernel"):
            d.tile = t + 1
            if Engine._plan_ok(d, e):
                built += 1
                assert e.nres > 0 or bool(e.residual) or bool(e.bn_mean), "built for a plain epilogue"
                continue
            refused += 1
            with pytest.raises(_lib.QnnError, match="not built"):
                eng.ops[idx](st)
        d.tile = 0
    torch.cuda.synchronize()
    assert built and refused


def test_dtab_general_geometry_bitwise(gpu):
    """the per-pixel border-class lookup (nclass > 1) and the non-DENSE instantiation
    of the table epilogue are exercised -- CIFAR ResNet-18's 3x3 general-chain convolutions (16 and
    32 input channels, zero-padded consumer outputs) with configurations 42 and 43 forced, bitwise
    against the module path.  (No model here has a stride-2 general-chain contraction: a block's
    strided conv is its first, whose epilogue is the code table -- refused by these configurations.)"""
    from qnn.engine import Engine
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    batch = 6
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 93)
    model = model.to(gpu)
    xg = x.to(gpu)
    feat = _module_feat(model, xg).permute(0, 2, 3, 1)
    covered = []
    for t in _lib.tile_ids("qconv_dtab_kernel"):
        eng = Engine(model, batch=batch, graph=False, tile=t)
        forced = [(dd, ee) for (k, _), (_n, dd, ee) in zip(eng.tiles, eng.convs) if dd.tile == t + 1]
        covered += [(t, dd.kh, ee.nclass, ee.code0_pad) for dd, ee in forced]
        for rep in range(2):
            eng(xg)
            torch.cuda.synchronize()
            assert torch.equal(eng.head_input, feat), f"configuration {t} run {rep}: engine != module path"
    # configuration 42 (four pixel tiles per wave) takes K <= 128 only; 43 the 16-channel 3x3s (K 144)
    assert any(kh == 3 and ncls > 1 for _t, kh, ncls, _p in covered), f"no 3x3 with border classes forced: {covered}"
    assert any(pad > 0 for *_x, pad in covered), f"no padded consumer output: {covered}"
