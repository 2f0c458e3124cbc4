"""GPU parity of the HIP path against the oracle and the reference's golden outputs.

Tolerances:
  * quantizer outputs / codes / packed weights: bit-exact;
  * one layer on identical inputs: max|dy| <= 1e-5 * max|y_ref| + 1e-6 (the int32
    contraction is exact; the error is fp32 epilogue rounding vs oneDNN's fp32 sum);
  * every layer inside each model, teacher-forced on the input the GPU forward fed
    it: the per-layer bar above (RangeBN bit-exact);
  * whole model: max|dlogit| <= max(3e-2 * max|logit_ref|, 1.5 * drift64), where
    drift64 is the reference's own logit change when its contraction runs in fp64
    (a 1-ulp conv difference can flip a downstream round());
    top-1 equal wherever the reference's top-1 margin exceeds 2 * drift64.
"""
import glob
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import GOLDEN, load_fixture
from fixtures_util import build_layer, build_model, e2e_tolerance, oracle_fp64_drift, oracle_layer
from oracle import qnn_oracle as O
from qnn import _lib, synthetic
from qnn.quantize import QConv2d, QLinear, RangeBN, quantize, set_measure_mode

pytestmark = pytest.mark.gpu

LAYER_TOL = 1e-5
LAYERS = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "layer_*.npz")))
MODELS = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "model_*.npz")))


def _close(y, ref, tol=LAYER_TOL):
    y, ref = y.detach().float().cpu(), ref.detach().float().cpu()
    assert y.shape == ref.shape
    err = (y - ref).abs().max().item()
    bound = tol * ref.abs().max().item() + 1e-6
    assert err <= bound, f"max|dy|={err:.3e} > {bound:.3e} (max|y|={ref.abs().max().item():.3e})"
    return err


# ------------------------------------------------------------------ quantizer: bit-exact
def test_fake_quant_float_range_kat(gpu):
    d = load_fixture("quantize_kat")
    i = 0
    while f"float/{i}/x" in d:
        x = torch.from_numpy(d[f"float/{i}/x"]).to(gpu)
        mn, mx = d[f"float/{i}/range"]
        y = quantize(x, 8, float(mn), float(mx)).cpu().numpy()
        np.testing.assert_array_equal(y.view(np.uint32), d[f"float/{i}/y"].view(np.uint32))
        i += 1


def test_fake_quant_tensor_and_none_kat(gpu):
    d = load_fixture("quantize_kat")
    i = 0
    while f"tensor/{i}/x" in d:
        w = torch.from_numpy(d[f"tensor/{i}/x"]).to(gpu)
        sh = (w.shape[0],) + (1,) * (w.dim() - 1)
        y = quantize(w, 8, w.flatten(1).min(-1)[0].view(sh), w.flatten(1).max(-1)[0].view(sh))
        np.testing.assert_array_equal(y.cpu().numpy(), d[f"tensor/{i}/y"])
        i += 1
    j = 0
    while f"none/{j}/x" in d:
        y = quantize(torch.from_numpy(d[f"none/{j}/x"]).to(gpu), num_bits=8)
        np.testing.assert_array_equal(y.cpu().numpy(), d[f"none/{j}/y"])
        j += 1


@pytest.mark.parametrize("shape,c_pad,pad", [
    ((3, 24, 9, 11), 32, 1), ((2, 3, 33, 17), 16, 3),     # w % 4 != 0: one pixel per thread
    ((4, 64, 56, 56), 64, 0), ((2, 40, 12, 16), 48, 1),   # w % 4 == 0: 4 pixels per thread + the padding ring
    ((3, 24, 8, 20), 32, 2), ((2, 128, 28, 28), 128, 1), ((1, 5, 4, 4), 16, 3),
])
def test_activation_codes_padded_nhwc8(gpu, shape, c_pad, pad):
    N, C, H, W = shape
    x = synthetic.input_batch(shape, 5) * 2.0
    mn, mx = -1.5, 3.25
    hp, wp = H + 2 * pad, W + 2 * pad
    nbytes = N * hp * wp * c_pad
    q = torch.full((nbytes + 128,), 77, dtype=torch.int8, device=gpu)  # poisoned
    s = max((mx - mn) / 255.0, 1e-8)
    xd = x.to(gpu)
    _lib.call("qnn_quantize_nchw_to_nhwc8", _lib.ptr(xd), _lib.ptr(q), N, C, H, W, pad, c_pad, -mn, s, 255.0,
              _lib.stream_of(xd))
    got = q[:nbytes].cpu().numpy().astype(np.int32).reshape(N, hp, wp, c_pad)
    ref = O.quantize_codes_np(x.numpy(), mn, mx).astype(np.int32) - 128  # N C H W
    np.testing.assert_array_equal(got[:, pad:pad + H, pad:pad + W, :C], ref.transpose(0, 2, 3, 1))
    inner = np.zeros((N, hp, wp, c_pad), dtype=bool)
    inner[:, pad:pad + H, pad:pad + W, :C] = True
    assert np.all(got[~inner] == 0)                              # border + channel pad = code' 0
    assert np.all(q[nbytes:].cpu().numpy() == 0)                 # zero page


@pytest.mark.parametrize("H,W,pad,hz,wz", [
    (37, 30, 3, 21, 18),     # w % 4 != 0: one s2d pixel per thread
    (36, 32, 3, 20, 19),     # w % 4 == 0: two per thread (aligned float4 pairs), 7x7/2 stem padding, odd wz
    (36, 32, 1, 18, 17),     # MobileNet's 3x3/2 stem padding
    (40, 40, 2, 22, 22),     # even padding
    (224, 224, 3, 115, 115),  # the ResNet stem at 224 (one wave per s2d row)
    (224, 224, 1, 113, 113),  # the MobileNet stem at 224 (odd hz, wz)
    (12, 264, 3, 9, 135),    # more than 64 pairs per row: the grid-stride form
])
def test_activation_codes_space_to_depth(gpu, H, W, pad, hz, wz):
    N, C = 2, 3
    x = synthetic.input_batch((N, C, H, W), 6)
    mn, mx = -2.0, 2.5
    z = torch.full((N * hz * wz * 16 + 128,), 55, dtype=torch.int8, device=gpu)
    xd = x.to(gpu)
    _lib.call("qnn_quantize_nchw_to_s2d8", _lib.ptr(xd), _lib.ptr(z), N, C, H, W, pad, hz, wz, -mn,
              max((mx - mn) / 255.0, 1e-8), 255.0, _lib.stream_of(xd))
    got = z[: N * hz * wz * 16].cpu().numpy().astype(np.int32).reshape(N, hz, wz, 16)
    codes = O.quantize_codes_np(x.numpy(), mn, mx).astype(np.int32) - 128
    ref = np.zeros_like(got)
    for h2 in range(hz):
        for w2 in range(wz):
            for u in range(2):
                for v in range(2):
                    iy, ix = 2 * h2 + u - pad, 2 * w2 + v - pad
                    if 0 <= iy < H and 0 <= ix < W:
                        ref[:, h2, w2, (2 * u + v) * C:(2 * u + v + 1) * C] = codes[:, :, iy, ix]
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("shape,s2d", [((64, 64, 3, 3), 0), ((40, 24, 3, 3), 0), ((64, 3, 7, 7), 0),
                                       ((1000, 512, 1, 1), 0), ((64, 3, 7, 7), 2), ((32, 3, 3, 3), 2)])
def test_weight_pack_bitexact(gpu, shape, s2d):
    w = torch.from_numpy(synthetic.normal(shape, 9, 0, 0.05))
    w[1] = 0.25  # constant channel -> scale floor
    cout, cin, kh, kw = shape
    cin_pad = 16 if s2d else max(16, 1 << (cin - 1).bit_length())
    pkh, pkw = ((kh + 1) // 2, (kw + 1) // 2) if s2d else (kh, kw)
    cout_pad = (cout + 127) // 128 * 128
    kpad = (pkh * pkw * cin_pad + 127) // 128 * 128
    wd = w.to(gpu)
    wq = torch.full((cout_pad, kpad), 99, dtype=torch.int8, device=gpu)
    f = lambda *s: torch.empty(s, dtype=torch.float32, device=gpu)
    s_w, b_w, tap, what, wmin, wmax = f(cout), f(cout), f(cout, kh * kw), f(cout, cin * kh * kw), f(cout), f(cout)
    _lib.call("qnn_pack_weight_i8", _lib.ptr(wd), cout, cin, kh, kw, cin_pad, cout_pad, s2d, 255.0, None, None,
              _lib.ptr(wq), _lib.ptr(s_w), _lib.ptr(b_w), _lib.ptr(tap), _lib.ptr(what), _lib.ptr(wmin),
              _lib.ptr(wmax), _lib.stream_of(wd))
    lo, hi = O.weight_ranges(w)
    codes = (O.codes_tensor_range(w, lo, hi).to(torch.int32) - 128).numpy()      # [cout][cin][kh][kw]
    packed = wq.cpu().numpy().astype(np.int32)
    ref = np.zeros_like(packed)
    for r in range(kh):
        for sx in range(kw):
            for ci in range(cin):
                if s2d:
                    a, u, b, v = r // 2, r % 2, sx // 2, sx % 2
                    col = (a * pkw + b) * cin_pad + (2 * u + v) * cin + ci
                else:
                    col = (r * kw + sx) * cin_pad + ci
                ref[:cout, col] = codes[:, ci, r, sx]
    np.testing.assert_array_equal(packed, ref)
    w_hat = O.uniform_quantize(w, 8, lo, hi)
    np.testing.assert_array_equal(what.cpu().numpy(), w_hat.reshape(cout, -1).numpy())
    np.testing.assert_array_equal(wmin.cpu().numpy(), lo.reshape(-1).numpy())
    np.testing.assert_array_equal(wmax.cpu().numpy(), hi.reshape(-1).numpy())
    ref_tap = w_hat.double().sum(1).reshape(cout, kh * kw).float()
    torch.testing.assert_close(tap.cpu(), ref_tap, rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------------ layers vs golden + oracle
@pytest.mark.parametrize("name", LAYERS)
def test_layer_vs_reference_golden(gpu, name):
    d = load_fixture("layer_" + name)
    wrap, m, x = build_layer(d)
    wrap = wrap.to(gpu)
    with torch.no_grad():
        y = wrap(x.to(gpu))
    _close(y, torch.from_numpy(d["y"]))
    if isinstance(m, (QConv2d, QLinear)):
        # weight_min/max buffers are refreshed as the reference does
        ref_lo, ref_hi = O.weight_ranges(m.weight.detach().cpu())
        assert torch.equal(m.weight_min.cpu(), ref_lo) and torch.equal(m.weight_max.cpu(), ref_hi)


CONV_CASES = [
    # (cin, cout, k, stride, pad, groups, bias, N, H, W)
    (256, 256, 3, 1, 1, 1, False, 4, 14, 14),     # headline ResNet-50 layer3 3x3
    (64, 64, 3, 1, 1, 1, False, 2, 56, 56),       # ResNet-18 layer1
    (3, 64, 7, 2, 3, 1, False, 2, 224, 224),      # stem
    (1024, 256, 1, 1, 0, 1, False, 4, 14, 14),    # bottleneck 1x1 reduce
    (512, 2048, 1, 1, 0, 1, False, 2, 7, 7),      # bottleneck 1x1 expand (cout 2048)
    (256, 512, 1, 2, 0, 1, False, 4, 14, 14),     # strided downsample
    (96, 80, 3, 2, 1, 1, True, 3, 15, 13),        # ragged, odd sizes, bias
    (128, 128, 3, 2, 1, 128, True, 4, 28, 28),    # depthwise s2
    (32, 32, 3, 1, 1, 32, True, 2, 112, 112),     # depthwise s1 (mobilenet first block)
    (1024, 1024, 3, 1, 1, 1024, False, 3, 7, 7),  # depthwise, 1024 channels, 7x7
    (16, 16, 3, 2, 1, 16, True, 5, 15, 13),       # depthwise, ragged stride 2
    (48, 48, 3, 1, 1, 48, False, 2, 9, 9),        # depthwise, channels not a power of two
    (24, 24, 3, 1, 1, 24, True, 2, 10, 10),       # depthwise, c % 8 == 0 but not % 16
    (32, 32, 3, 1, 1, 32, False, 3, 30, 30),      # depthwise, 30x30
    (64, 64, 3, 2, 1, 64, True, 2, 57, 57),       # depthwise, odd extent stride 2
]


@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_vs_oracle(gpu, case):
    cin, cout, k, st, pd, g, bias, N, H, W = case
    m = QConv2d(cin, cout, k, stride=st, padding=pd, groups=g, bias=bias, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 3)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(2.75)
    wrap.eval()
    x = synthetic.input_batch((N, cin, H, W), 17, relu=True) * 1.1
    sd = {kk: v.clone() for kk, v in wrap.state_dict().items()}
    ref = O.qconv2d(x, sd["0.weight"], sd.get("0.bias"), st, pd, 1, g, (0.0, 2.75))
    with torch.no_grad():
        y = wrap.to(gpu)(x.to(gpu))
    _close(y, ref)


def test_linear_vs_oracle(gpu):
    m = QLinear(2048, 1000, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 4)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(1.5)
    wrap.eval()
    x = synthetic.input_batch((37, 2048), 18, relu=True) * 0.6
    sd = {kk: v.clone() for kk, v in wrap.state_dict().items()}
    ref = O.qlinear(x, sd["0.weight"], sd["0.bias"], (0.0, 1.5))
    with torch.no_grad():
        y = wrap.to(gpu)(x.to(gpu))
    _close(y, ref)


def test_rangebn_bitexact_given_input(gpu):
    d = load_fixture("layer_rbn_32")
    wrap, m, x = build_layer(d)
    ref = oracle_layer(O, d, wrap, x)
    with torch.no_grad():
        y = wrap.to(gpu)(x.to(gpu))
    np.testing.assert_array_equal(y.cpu().numpy(), ref.numpy())


# ------------------------------------------------------------------ models end to end
@pytest.mark.parametrize("name", MODELS)
def test_model_layers_teacher_forced(gpu, name):
    """Every QConv2d / QLinear / RangeBN of the model, on the exact input it sees
    inside the GPU forward, against the oracle layer: the tight per-layer bar in
    model context (RangeBN bit-exact given its input)."""
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    model = model.to(gpu)
    seen = []
    hooks = [m.register_forward_hook(lambda m, i, o: seen.append((m, i[0].detach().cpu(), o.detach().cpu())))
             for m in model.modules() if isinstance(m, (QConv2d, QLinear, RangeBN))]
    with torch.no_grad():
        model(x.to(gpu))
    for h in hooks:
        h.remove()
    assert len(seen) > 20
    worst, worst_flip, flips = 0.0, 0.0, []
    for i, (m, xin, yout) in enumerate(seen):
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        rng = O.measure_range(sd, "quantize_input.")
        if isinstance(m, RangeBN):
            ref = O.rangebn(xin, sd["running_mean"], sd["running_var"], sd["weight"], sd["bias"], rng)
            assert torch.equal(yout, ref)
            continue
        if isinstance(m, QLinear):
            ref = O.qlinear(xin, sd["weight"], sd.get("bias"), rng)
        else:
            ref = O.qconv2d(xin, sd["weight"], sd.get("bias"), m.stride, m.padding, 1, m.groups, rng)
        worst = max(worst, _close(yout, ref) / ref.abs().max().item())
        # fraction of the consumer's activation codes that the fp32 epilogue
        # rounding flips (the conv output feeds the next RangeBN's quantizer directly)
        if i + 1 < len(seen) and isinstance(seen[i + 1][0], RangeBN) and torch.equal(seen[i + 1][1], yout):
            bsd = {k: v.detach().cpu() for k, v in seen[i + 1][0].state_dict().items()}
            lo, hi = O.measure_range(bsd, "quantize_input.")
            qg = O.quantize_codes_np(yout.numpy(), lo, hi)
            qr = O.quantize_codes_np(ref.numpy(), lo, hi)
            frac = float((qg != qr).mean())
            flips.append(frac)
            worst_flip = max(worst_flip, frac)
    print(f"{name}: {len(seen)} layers, worst max|dy|/max|y| = {worst:.2e}; flipped consumer codes per layer: "
          f"max {worst_flip:.2e}, mean {np.mean(flips) if flips else 0.0:.2e} over {len(flips)} conv->RangeBN pairs")
    assert flips, "no conv -> RangeBN pair found"
    assert worst_flip <= 1e-3, f"flipped-code fraction {worst_flip:.2e} > 1e-3"


@pytest.mark.parametrize("name", MODELS)
def test_model_vs_reference_golden(gpu, name):
    """Statistical end-to-end bar: within 1.5x the reference's own fp64-vs-fp32
    contraction drift (floor 3%), top-1 equal wherever the reference's own top-1
    margin exceeds that drift."""
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    ref = torch.from_numpy(d["logits"])
    drift64, _ = oracle_fp64_drift(O, sd, x, d["config"]["factory"], d["config"]["kw"], ref)
    with torch.no_grad():
        logits = model.to(gpu)(x.to(gpu)).cpu()
    err = (logits - ref).abs().max().item()
    tol = e2e_tolerance(ref, drift64)
    assert err <= tol, (err, tol, drift64)
    top2 = ref.topk(2, dim=1).values
    decisive = (top2[:, 0] - top2[:, 1]) > 2 * drift64
    assert torch.equal(logits.argmax(1)[decisive], ref.argmax(1)[decisive])


# ------------------------------------------------------------------ behaviour
def test_cpu_input_fails_loudly():
    m = QConv2d(16, 16, 3, padding=1).eval()
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.randn(1, 16, 8, 8))


def test_per_channel_false_raises_like_reference(gpu):
    m = QConv2d(16, 16, 3, padding=1, per_channel=False).to(gpu).eval()
    with pytest.raises(TypeError):
        m(torch.randn(1, 16, 8, 8, device=gpu))


def test_measure_mode_is_float_conv_and_calibrates(gpu):
    m = QConv2d(16, 8, 3, padding=1).to(gpu)
    wrap = nn.Sequential(m)
    set_measure_mode(wrap, True)
    wrap.train()
    x = torch.randn(4, 16, 8, 8, device=gpu)
    y = wrap(x)
    torch.testing.assert_close(y, torch.nn.functional.conv2d(x, m.weight, m.bias, 1, 1))
    lo = x.view(4, -1).min(-1)[0].mean()
    assert m.quantize_input.num_measurements.item() == 1
    torch.testing.assert_close(m.quantize_input.running_min, lo.view(1))  # first update: momentum 0/(0+1)


def test_pack_cache_tracks_weight_updates(gpu):
    m = QConv2d(32, 32, 3, padding=1, bias=False).to(gpu).eval()
    m.quantize_input.running_min.fill_(-1.0)
    m.quantize_input.running_max.fill_(1.0)
    x = torch.randn(2, 32, 8, 8, device=gpu)
    y1 = m(x)
    with torch.no_grad():
        m.weight.mul_(-1.0)
    y2 = m(x)
    assert not torch.allclose(y1, y2)
    ref = O.qconv2d(x.cpu(), m.weight.detach().cpu(), None, 1, 1, 1, 1, (-1.0, 1.0))
    _close(y2, ref)
