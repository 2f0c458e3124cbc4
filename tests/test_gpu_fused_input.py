"""The drop-in QConv2d forward with the input quantizer fused into the convolution.

qnn_qconv2d_fwd_nchw_f32 (include/qnn.h) reads the module's fp32 NCHW input and quantizes it
into the persistent-band kernel's LDS bands; the reference's QConv2d.forward
(/root/reference/models/modules/quantize.py:314-354) quantizes the input, then convolves, which
is the two-launch path here (qnn_quantize_nchw_to_nhwc8 + qnn_qconv2d_fwd).  Both must give the
bitwise same output: every persistent-band configuration that fits, strides 1 and 2, ragged
channel counts (cin < cp), bias, inputs outside the calibrated range (clamped codes), batches
whose last band runs past the batch; a layer no configuration fits falls back to two launches.
"""
import pytest
import torch
import torch.nn as nn

from oracle import qnn_oracle as O
from qnn import _lib, synthetic
from qnn.quantize import QConv2d

pytestmark = pytest.mark.gpu

PB_IDS = _lib.tile_ids("qconv_pb_kernel")

# (cin, cout, stride, N, H, W, bias)
CASES = [
    (64, 64, 1, 2, 56, 56, False),     # ResNet-18 layer 1
    (64, 128, 2, 3, 56, 56, False),    # ResNet-18 layer-2 entry (stride 2)
    (128, 128, 1, 2, 28, 28, False),   # ResNet-18 layer 2
    (48, 64, 1, 2, 20, 20, True),      # ragged channels (cp 64), bias
    (64, 64, 1, 5, 13, 11, False),     # odd geometry, ragged last band
    (100, 32, 2, 3, 17, 15, True),     # cp 128, stride 2, odd
]


def _layer(cin, cout, st, N, H, W, bias, seed=7):
    m = QConv2d(cin, cout, 3, stride=st, padding=1, bias=bias, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, seed)
    m.quantize_input.running_min.fill_(-0.25)
    m.quantize_input.running_max.fill_(2.5)
    wrap.eval()
    # outside [min, max] on both sides: the clamped codes 0 and qmax occur
    x = synthetic.input_batch((N, cin, H, W), seed + 1, relu=False) * 1.6 + 0.4
    return wrap, x


def _fwd(wrap, x, fused, tile=0):
    m = wrap[0]
    m.qnn_fused_input, m.qnn_fused_tile = fused, tile
    try:
        with torch.no_grad():
            y = wrap(x).clone()
        return y, m._last_fused
    finally:
        m.qnn_fused_input, m.qnn_fused_tile = None, 0


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}-s{c[2]}-n{c[3]}-{c[4]}x{c[5]}" for c in CASES])
def test_fused_input_bitwise_vs_two_launches(gpu, case):
    wrap, x = _layer(*case)
    wrap, xg = wrap.to(gpu), x.to(gpu)
    ref, f0 = _fwd(wrap, xg, False)
    assert not f0
    y, f1 = _fwd(wrap, xg, True)
    assert f1, "no persistent-band configuration took the fp32 input"
    assert torch.equal(y, ref)
    ran = 0
    for k in PB_IDS:
        yk, fk = _fwd(wrap, xg, True, tile=k + 1)
        if fk:
            ran += 1
            assert torch.equal(yk, ref), f"configuration {k}"
    assert ran >= 1


def test_fused_input_vs_oracle(gpu):
    cin, cout, st, N, H, W, bias = CASES[3]
    wrap, x = _layer(cin, cout, st, N, H, W, bias)
    sd = {k: v.clone() for k, v in wrap.state_dict().items()}
    ref = O.qconv2d(x, sd["0.weight"], sd.get("0.bias"), st, 1, 1, 1, (-0.25, 2.5))
    y, fused = _fwd(wrap.to(gpu), x.to(gpu), True)
    assert fused
    y, ref = y.cpu(), ref.float()
    err = (y - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item() + 1e-6


def test_fused_input_falls_back(gpu):
    """256 input channels: no persistent-band configuration; the two-launch path runs."""
    wrap, x = _layer(256, 64, 1, 2, 14, 14, False)
    wrap, xg = wrap.to(gpu), x.to(gpu)
    y, fused = _fwd(wrap, xg, True)
    assert not fused
    ref, _ = _fwd(wrap, xg, False)
    assert torch.equal(y, ref)


def test_fused_input_misaligned_view_falls_back(gpu):
    """A contiguous fp32 input at a 4-byte (not 16-byte) offset: the one-launch entry declines it
    (QNN_ERR_UNSUPPORTED) and the two-launch path runs, bitwise the same output."""
    wrap, x = _layer(*CASES[0])
    wrap, xg = wrap.to(gpu), x.to(gpu)
    ref, _ = _fwd(wrap, xg, False)
    buf = torch.empty(xg.numel() + 4, dtype=torch.float32, device=gpu)
    xm = buf[1:1 + xg.numel()].view_as(xg)
    xm.copy_(xg)
    assert xm.is_contiguous() and xm.data_ptr() % 16 != 0
    y, fused = _fwd(wrap, xm, True)
    assert not fused
    assert torch.equal(y, ref)


def test_spin_timeout_raises_device_error(gpu):
    """A persistent-band wave that gives up a bounded hand-off wait raises QNN_DEVERR_PB_SPIN in
    the device error word (forced here by a spin bound of 0); with the default bound the word stays
    clear and the output is the two-launch path's.  Batch 24: every block walks several bands, so
    its waves wait on one another's hand-offs."""
    wrap, x = _layer(64, 64, 1, 24, 56, 56, False)
    wrap, xg = wrap.to(gpu), x.to(gpu)
    ref, _ = _fwd(wrap, xg, False)
    assert _lib.device_errors() == 0
    _lib.call("qnn_debug_set_spin_limit", 0)
    try:
        _, fused = _fwd(wrap, xg, True)
        assert fused
        flags = _lib.device_errors()
    finally:
        _lib.call("qnn_debug_set_spin_limit", -1)
    assert flags & _lib.DEVERR_PB_SPIN, f"device error word {flags:#x}"
    y, fused = _fwd(wrap, xg, True)
    assert fused and _lib.device_errors() == 0
    assert torch.equal(y, ref)
