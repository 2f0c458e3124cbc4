"""Fused depthwise kernel (MobileNet's depthwise QConv2d + RangeBN + ReLU + the pointwise
consumer's quantizer, include/qnn.h qnn_dwconv_fused).

The 3x3 fast kernel (dwconv3_kernel: 4 channels x a 2 x 4 (stride 2: 2 x 2) pixel block per
thread, register weights, division-free quantizers, out-of-image taps masked to an exact
+0 in the code-table kernels) restates the generic kernel's arithmetic op for
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
    (3, 17, 36, 1, True, True),    # odd output height (a row pair's second row past the map), c/4 = 9
    (2, 10, 20, 2, False, True),   # stride 2, ho = 5: the last row pair half outside
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


@pytest.mark.parametrize("n,h,c,s,with_bias", [
    (2, 14, 32, 1, True),
    (3, 13, 64, 2, True),
    (2, 7, 1024, 1, True),       # eight 128-channel slices
    (4, 28, 256, 2, False),
    (2, 56, 128, 1, True),
    (1, 112, 32, 1, True),
    (2, 29, 512, 2, True),       # odd extent, stride 2, four slices
    (1, 15, 96, 1, False),       # one slice of 96 (c/8 = 12 does not divide 256)
])
def test_dwconv_lut_equals_evaluated_bitwise(gpu, n, h, c, s, with_bias):
    """qnn_dwconv_fused_lut (RangeBN -> ReLU -> consumer quantizer looked up in the
    qnn_bn_code_lut table, channel slices of <= 128 in LDS) writes bitwise the codes of the
    evaluated chain (qnn_dwconv_fused), pad columns / rows of the consumer buffer untouched."""
    g = torch.Generator().manual_seed(2000 + c + h)
    k, pad = 3, 1
    w = h
    ho = (h + 2 * pad - k) // s + 1
    wo = ho
    cp = c
    hp, wp = h + 2 * pad, w + 2 * pad
    xc = torch.zeros((n, hp, wp, cp), dtype=torch.int8)
    xc[:, pad:pad + h, pad:pad + w, :c] = torch.randint(-128, 128, (n, h, w, c), generator=g, dtype=torch.int8)
    xmin, xs = -0.75, 3.1 / 255
    wt = (torch.randn((k * k, c), generator=g) * 0.3).float().to(gpu)
    bias = (torch.randn(c, generator=g) * 0.1).float().to(gpu) if with_bias else None
    vecs = [torch.randn(c, generator=g) * 0.05, torch.rand(c, generator=g) + 0.5,
            torch.rand(c, generator=g) * 2 - 0.5, torch.randn(c, generator=g) * 0.1]  # some wq < 0
    vecs = [v.float().to(gpu) for v in vecs]
    bn = _lib.BnParams(*[_lib.ptr(v) for v in vecs], 0.9, -0.9, 2.2 / 255, 255.0)
    xg = xc.to(gpu)
    st = _lib.stream_of(xg)
    geom = (n, h, w, pad, hp, wp, cp, c, k, s, ho, wo, xmin, xs)
    outs = []
    for use_lut in (False, True):
        oc = torch.full((n, ho + 2, wo + 2, cp), 77, dtype=torch.int8, device=gpu)
        code = _lib.CodeOut(_lib.ptr(oc), cp, 1, ho + 2, wo + 2, 0.2, 1.7 / 255, 255.0)
        if use_lut:
            lut = torch.empty((c, 256), dtype=torch.int8, device=gpu)
            _lib.call("qnn_bn_code_lut", ctypes.byref(bn), c, 1, ctypes.byref(code), _lib.ptr(lut), st)
            _lib.call("qnn_dwconv_fused_lut", _lib.ptr(xg), n, h, w, pad, hp, wp, cp, c, _lib.ptr(wt), k, k, s, s,
                      ho, wo, xmin, xs, None if bias is None else _lib.ptr(bias), ctypes.byref(bn), _lib.ptr(lut),
                      ctypes.byref(code), st)
            torch.cuda.synchronize()
        else:
            _run(xg, geom, wt, bias, bn, 1, None, code, False, st)
        outs.append(oc.cpu())
    assert torch.equal(outs[0], outs[1]), int((outs[0] != outs[1]).sum())
    assert (outs[1][:, 0] == 77).all() and (outs[1][:, :, 0] == 77).all()  # the consumer's padding untouched


def test_dwconv_lut_refuses_unsupported(gpu):
    """Shapes the table kernel is not built for are argument errors, never a silent substitute."""
    c, n, h = 192, 1, 8  # above 128 channels and not a multiple of 128
    x = torch.zeros((n, h + 2, h + 2, c), dtype=torch.int8, device=gpu)
    wt = torch.zeros((9, c), device=gpu)
    vecs = [torch.ones(c, device=gpu) for _ in range(4)]
    bn = _lib.BnParams(*[_lib.ptr(v) for v in vecs], 0.9, -0.9, 2.2 / 255, 255.0)
    oc = torch.zeros((n, h, h, c), dtype=torch.int8, device=gpu)
    code = _lib.CodeOut(_lib.ptr(oc), c, 0, h, h, 0.2, 1.7 / 255, 255.0)
    lut = torch.zeros((c, 256), dtype=torch.int8, device=gpu)
    with pytest.raises(_lib.QnnError, match="qnn_dwconv_fused_lut"):
        _lib.call("qnn_dwconv_fused_lut", _lib.ptr(x), n, h, h, 1, h + 2, h + 2, c, c, _lib.ptr(wt), 3, 3, 1, 1, h, h,
                  -0.75, 0.01, None, ctypes.byref(bn), _lib.ptr(lut), ctypes.byref(code), _lib.stream_of(x))


def test_dwconv_lut_chunked_past_2gib(gpu):
    """Inputs past 2 GiB: the 3x3 kernel addresses an input by 32-bit buffer offsets, so the host
    launches it over chunks of images (here 4 + 1 images of 514 MB); the codes match the generic
    kernel's evaluated chain bitwise, the consumer's padding untouched."""
    n, h, c, s = 5, 1000, 512, 1
    k, pad = 3, 1
    w, ho, wo, cp = h, h, h, c
    hp, wp = h + 2 * pad, w + 2 * pad
    assert n * hp * wp * cp >= 1 << 31
    g = torch.Generator(device=gpu).manual_seed(77)
    xg = torch.zeros((n, hp, wp, cp), dtype=torch.int8, device=gpu)
    xg[:, pad:pad + h, pad:pad + w, :] = torch.randint(-128, 128, (n, h, w, c), generator=g, dtype=torch.int8,
                                                        device=gpu)
    xmin, xs = -0.75, 3.1 / 255
    wt = torch.randn((k * k, c), generator=g, device=gpu) * 0.3
    vecs = [torch.randn(c, generator=g, device=gpu) * 0.05, torch.rand(c, generator=g, device=gpu) + 0.5,
            torch.rand(c, generator=g, device=gpu) * 2 - 0.5, torch.randn(c, generator=g, device=gpu) * 0.1]
    bn = _lib.BnParams(*[_lib.ptr(v) for v in vecs], 0.9, -0.9, 2.2 / 255, 255.0)
    st = _lib.stream_of(xg)
    outs = []
    for use_lut in (False, True):
        oc = torch.full((n, ho + 2, wo + 2, cp), 77, dtype=torch.int8, device=gpu)
        code = _lib.CodeOut(_lib.ptr(oc), cp, 1, ho + 2, wo + 2, 0.2, 1.7 / 255, 255.0)
        if use_lut:
            lut = torch.empty((c, 256), dtype=torch.int8, device=gpu)
            _lib.call("qnn_bn_code_lut", ctypes.byref(bn), c, 1, ctypes.byref(code), _lib.ptr(lut), st)
            _lib.call("qnn_dwconv_fused_lut", _lib.ptr(xg), n, h, w, pad, hp, wp, cp, c, _lib.ptr(wt), k, k, s, s,
                      ho, wo, xmin, xs, None, ctypes.byref(bn), _lib.ptr(lut), ctypes.byref(code), st)
        else:
            _lib.call("qnn_dwconv_fused_generic", _lib.ptr(xg), n, h, w, pad, hp, wp, cp, c, _lib.ptr(wt), k, k, s,
                      s, ho, wo, xmin, xs, None, ctypes.byref(bn), 1, None, ctypes.byref(code), st)
        torch.cuda.synchronize()
        outs.append(oc)
    assert torch.equal(outs[0], outs[1]), int((outs[0] != outs[1]).sum())
    assert bool((outs[1][:, 0] == 77).all()) and bool((outs[1][:, :, 0] == 77).all())
