"""Fused depthwise kernel (MobileNet's depthwise QConv2d + RangeBN + ReLU + the pointwise
consumer's quantizer, include/qnn.h qnn_dwconv_fused).

The 3x3 fast kernel (dwconv3_kernel: 8 channels x 4 pixels per thread, register
weights, division-free quantizers) restates the generic kernel's arithmetic op for
op, so both must agree BITWISE on every output (fp32 and codes) — over strides 1/2,
larger maps and
ragged widths (wo not a multiple of 4), channel counts whose c/8 does not divide 256,
with and without bias / RangeBN.  The fp32 output is also held to the per-layer bar
against an fp64 restatement of the reference's depthwise conv (quantize.py:343,
groups == cin) on the dequantized codes.
"""
import ctypes

import numpy as np
import pytest
import torch

from qnn import _lib

pytestmark = pytest.mark.gpu


def _run(xcodes, geom, wt, bias, bn, relu, out_f32, code, generic, st):
    n, h, w, pad, hp, wp, cp, c, k, s, ho, wo, xmin, xs = geom
    _lib.call("qnn_dwconv_fused_generic" if generic else "qnn_dwconv_fused", _lib.ptr(xcodes), n, h, w, pad, hp, wp,
              cp, c, _lib.ptr(wt), k, k, s, s, ho, wo, xmin, xs, None if bias is None else _lib.ptr(bias),
              None if bn is None else ctypes.byref(bn), relu, _lib.ptr(out_f32), ctypes.byref(code), st)
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,h,c,s,with_bias,with_bn", [
    (2, 14, 32, 1, True, True),
    (3, 13, 64, 2, True, True),
    (2, 7, 1024, 1, True, True),
    (1, 9, 24, 1, False, False),   # c/8 = 3 does not divide 256; wo = 9
    (2, 11, 40, 2, True, False),   # ragged, stride 2
    (4, 28, 256, 2, False, True),
    (2, 56, 128, 1, True, True),
    (1, 112, 32, 1, True, True),
    (2, 29, 64, 2, True, True),    # odd extent, stride 2
    (1, 15, 96, 1, False, True),
])
def test_dwconv_fast_equals_generic_bitwise(gpu, n, h, c, s, with_bias, with_bn):
    g = torch.Generator().manual_seed(1000 + c + h)
    k, pad = 3, 1
    w = h
    ho = (h + 2 * pad - k) // s + 1
    wo = ho
    cp = c if c % 16 == 0 else (c + 15) // 16 * 16
    hp, wp = h + 2 * pad, w + 2 * pad
    xc = torch.zeros((n, hp, wp, cp), dtype=torch.int8)
    xc[:, pad:pad + h, pad:pad + w, :c] = torch.randint(-128, 128, (n, h, w, c), generator=g, dtype=torch.int8)
    xmin, xs = -0.75, 3.1 / 255
    wt = (torch.randn((k * k, c), generator=g) * 0.3).float()
    bias = (torch.randn(c, generator=g) * 0.1).float() if with_bias else None
    keep = []
    bn = None
    if with_bn:
        vecs = [torch.randn(c, generator=g) * 0.05, torch.rand(c, generator=g) + 0.5,
                torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1]
        vecs = [v.float().to(gpu) for v in vecs]
        keep += vecs
        bn = _lib.BnParams(*[_lib.ptr(v) for v in vecs], 0.9, -0.9, 2.2 / 255, 255.0)
    xg, wg = xc.to(gpu), wt.to(gpu)
    bg = None if bias is None else bias.to(gpu)
    st = _lib.stream_of(xg)
    outs = []
    for generic in (True, False):
        of = torch.full((n, ho, wo, c), float("nan"), device=gpu)
        oc = torch.zeros((n, ho + 2, wo + 2, cp), dtype=torch.int8, device=gpu)
        code = _lib.CodeOut(_lib.ptr(oc), cp, 1, ho + 2, wo + 2, 0.2, 1.7 / 255, 255.0)
        geom = (n, h, w, pad, hp, wp, cp, c, k, s, ho, wo, xmin, xs)
        _run(xg, geom, wg, bg, bn, 1, of, code, generic, st)
        outs.append((of.cpu(), oc.cpu()))
    (f0, c0), (f1, c1) = outs
    assert torch.isfinite(f1).all()
    assert torch.equal(f0, f1), (f0 - f1).abs().max()
    assert torch.equal(c0, c1)
    if not with_bn:  # conv (+bias) -> ReLU against fp64 on the same dequantized codes
        q = (xc[:, pad:pad + h, pad:pad + w, :c].to(torch.int32) + 128).to(torch.float32)
        xhat = (q * xs + xmin).double().permute(0, 3, 1, 2)
        wk = wt.double().t().reshape(c, 1, k, k)
        ref = torch.nn.functional.conv2d(xhat, wk, None if bias is None else bias.double(), stride=s, padding=pad,
                                         groups=c).clamp_min(0).permute(0, 2, 3, 1)
        err = (f1.double() - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item() + 1e-6, err
