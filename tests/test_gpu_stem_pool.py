"""The fused stem conv + max-pool launch (qnn_qconv2d_maxpool_fwd, csrc/stem_pool.hip).

Bitwise against the two-launch path it replaces -- qnn_qconv2d_fwd writing the stem's
RangeBN input codes, then qnn_maxpool_bn (resnet_quantized.py:140-143, :171-174;
quantize.py:461-462) -- on the ImageNet stem at 224x224 and at sizes whose pooled height is
odd (the last row group of a block is partial), and inside the engine (ResNet-18 / -50):
fused and unfused engines produce the identical classifier input.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import load_fixture
from fixtures_util import build_model
from qnn import _lib, synthetic
from qnn.quantize import QConv2d, RangeBN, _qmax, float_scale

pytestmark = pytest.mark.gpu


def _stem(seed):
    conv = QConv2d(3, 64, 7, stride=2, padding=3, bias=False, num_bits_grad=8, biprecision=True)
    bn = RangeBN(64, num_bits=8, num_bits_grad=8)
    wrap = nn.Sequential(conv, bn)
    synthetic.init_params(wrap, seed)
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # both pool directions (sq * wq < 0 on some channels)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.2, 1.0)
    conv.quantize_input.running_min.fill_(-2.2)
    conv.quantize_input.running_max.fill_(2.6)
    bn.quantize_input.running_min.fill_(-3.0)
    bn.quantize_input.running_max.fill_(4.0)
    return wrap.eval()


def _run(wrap, x, dev, fused):
    conv, bn = wrap[0], wrap[1]
    N, _, H, W = x.shape
    st = _lib.stream_of(x)
    pk = conv._pack(s2d=True)
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    hz, wz = Ho + 3, Wo + 3
    mn, mx = conv.quantize_input._eval_range()
    s = float_scale(mn, mx, 8)
    nbytes = N * hz * wz * 16
    zq = torch.zeros(nbytes + 128, dtype=torch.int8, device=dev)
    _lib.call("qnn_quantize_nchw_to_s2d8", _lib.ptr(x), _lib.ptr(zq), N, 3, H, W, 3, hz, wz, -float(mn), s, 255.0, st)
    s32 = float(np.float32(s))
    g = conv._geometry(pk, H, W, 7, 7, 2, 2, 3, 3, Ho, Wo, dev)
    sxsw, sxbw, table = conv._epilogue(pk, g, (H, W), s32, 128.0 * s32 + float(np.float32(mn)), 7, 7)
    d = _lib.ConvDesc()
    d.n, d.cout, d.cout_pad, d.ho, d.wo, d.kpad = N, 64, pk.cout_pad, Ho, Wo, pk.kpad
    d.hp, d.wp, d.cp, d.zero_off = hz, wz, 16, nbytes
    d.kh, d.kw, d.sh, d.sw, d.kmask = 4, 4, 1, 1, pk.kmask.data_ptr()
    sq, wq, bq = bn._params(bn.running_var)
    bmn, bmx = bn.quantize_input._eval_range()
    b = _lib.BnParams(mean=bn.running_mean.data_ptr(), sq=sq.data_ptr(), wq=wq.data_ptr(), bq=bq.data_ptr(),
                      neg_min=-float(bmn), min=float(bmn), scale=float_scale(bmn, bmx, 8), qmax=_qmax(8))
    e = _lib.Epilogue()
    e.mode = 1
    e.sxsw, e.sxbw, e.table = sxsw.data_ptr(), sxbw.data_ptr(), table.data_ptr()
    e.hcls, e.wcls, e.nwc, e.nclass = g[0].data_ptr(), g[3].data_ptr(), g[5], g[2] * g[5]
    e.bn_mean, e.bn_sq, e.bn_wq, e.bn_bq = b.mean, b.sq, b.wq, b.bq
    e.bn_neg_min, e.bn_min, e.bn_scale, e.bn_qmax = b.neg_min, b.min, b.scale, b.qmax
    e.relu = 1
    Hp, Wp = (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1
    outs, luts = [], []
    for k, (lo, hi, pad) in enumerate(((-0.5, 3.5, 1), (0.0, 2.0, 0))):  # two consumers, padded and not
        buf = torch.full((N * (Hp + 2 * pad) * (Wp + 2 * pad) * 64 + 128,), 77, dtype=torch.int8, device=dev)
        co = _lib.CodeOut(ptr=buf.data_ptr(), cp=64, pad=pad, hp=Hp + 2 * pad, wp=Wp + 2 * pad, neg_min=-lo,
                          scale=float_scale(lo, hi, 8), qmax=255.0)
        lut = torch.empty((64, 256), dtype=torch.int8, device=dev)
        _lib.call("qnn_bn_code_lut", ctypes.byref(b), 64, 1, ctypes.byref(co), _lib.ptr(lut), st)
        outs.append((buf, co))
        luts.append(lut)
    ct = 2
    pcode = torch.full((-(-N * Hp * Wp // 32) * 32 * ct * 32,), 99, dtype=torch.uint8, device=dev)
    if fused:
        _lib.call("qnn_qconv2d_maxpool_fwd", _lib.ptr(zq), _lib.ptr(pk.wq), ctypes.byref(d), ctypes.byref(e), Hp, Wp,
                  _lib.ptr(pcode), _lib.ptr(luts[0]), ctypes.byref(outs[0][1]), _lib.ptr(luts[1]),
                  ctypes.byref(outs[1][1]), st)
    else:
        bncode = torch.empty((N, Ho, Wo, 64), dtype=torch.uint8, device=dev)
        e.out_bncode = bncode.data_ptr()
        _lib.call("qnn_qconv2d_fwd", _lib.ptr(zq), _lib.ptr(pk.wq), ctypes.byref(d), ctypes.byref(e), st)
        _lib.call("qnn_maxpool_bn", _lib.ptr(bncode), N, Ho, Wo, 64, 3, 2, 1, Hp, Wp, ctypes.byref(b), 1, None, 1,
                  _lib.ptr(pcode), _lib.ptr(luts[0]), ctypes.byref(outs[0][1]), _lib.ptr(luts[1]),
                  ctypes.byref(outs[1][1]), st)
    torch.cuda.synchronize()
    return pcode, outs[0][0], outs[1][0]


@pytest.mark.parametrize("N,H,W", [(4, 224, 224), (3, 98, 98), (2, 66, 90), (1, 30, 30)])
def test_stem_pool_bitwise_vs_two_launches(gpu, N, H, W):
    wrap = _stem(5).to(gpu)
    x = synthetic.input_batch((N, 3, H, W), 6).to(gpu)
    a = _run(wrap, x, gpu, fused=True)
    b = _run(wrap, x, gpu, fused=False)
    for name, u, v in zip(("pooled codes", "consumer 0 codes", "consumer 1 codes"), a, b):
        assert torch.equal(u, v), f"{name}: {int((u != v).sum())} bytes differ"


@pytest.mark.parametrize("fixture,batch", [("model_resnet18_imagenet", 128), ("model_resnet50_imagenet", 8)])
def test_engine_fused_stem_bitwise(gpu, fixture, batch):
    from qnn.engine import Engine
    d = load_fixture(fixture)
    model, _ = build_model(d)
    model = model.to(gpu)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 95).to(gpu)
    ef = Engine(model, batch=batch, autotune=False)
    eu = Engine(model, batch=batch, autotune=False, fuse_stem_pool=False)
    assert "qnn_qconv2d_maxpool_fwd" in ef.launch_names and "qnn_maxpool_bn" not in ef.launch_names
    assert "qnn_maxpool_bn" in eu.launch_names
    ef(x)
    eu(x)
    torch.cuda.synchronize()
    assert torch.equal(ef.head_input, eu.head_input)
    assert torch.equal(ef.logits, eu.logits)
