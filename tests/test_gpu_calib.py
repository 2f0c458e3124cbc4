"""GPU calibration statistics against the oracle's restatement.

qnn_measure_stats_f32 (QuantMeasure train branch, quantize.py:225-236) and
qnn_rangebn_stats_f32 (RangeBN train branch, :466-472) reduce in a fixed order with
fp64 accumulation; the reference (and the oracle, pinned bitwise to it by
tests/test_oracle_calib.py) reduces in fp32 torch order.  Bar: extrema exact, means and
std within CAL_TOL relative.  Then the module path's measure mode on the GPU reproduces
the reference-calibrated buffers of the layer fixtures to the same bar.
"""
import pytest
import torch
import torch.nn as nn

from conftest import fixture_buffers, load_fixture
from fixtures_util import build_model
from oracle import qnn_oracle as O
from qnn import synthetic
from qnn.quantize import QConv2d, QLinear, RangeBN, measure_stats, rangebn_stats, set_measure_mode

pytestmark = pytest.mark.gpu

CAL_TOL = 2e-6  # fp32 (reference order) vs fp64-accumulated, correctly rounded


def _close(a, b, tol=CAL_TOL):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    assert a.shape == b.shape
    err = (a - b).abs()
    bound = tol * b.abs().clamp_min(1.0)
    assert bool((err <= bound).all()), f"max err {err.max().item():.3e}"


SHAPES = [(16, 3, 224, 224), (2, 64, 56, 56), (128, 512, 7, 7), (3, 24, 9, 11), (4, 512), (1, 7), (256, 2048)]


@pytest.mark.parametrize("shape", SHAPES)
def test_measure_stats_vs_oracle(gpu, shape):
    x = synthetic.input_batch(shape, 31, relu=len(shape) == 4) * 1.7 - 0.2
    got = measure_stats(x.to(gpu))
    want = O.measure_stats(x)
    for g, w in zip(got[:2], want[:2]):
        _close(g, w)  # mean of per-sample extrema
    _close(got[2], want[2])
    if x.numel() > 1:
        _close(got[3], want[3])


@pytest.mark.parametrize("shape,chunks", [((16, 64, 56, 56), 16), ((4, 32, 8, 8), 16), ((2, 512, 7, 7), 2),
                                          ((8, 100), 8), ((3, 24, 9, 11), 3)])
def test_rangebn_stats_vs_oracle(gpu, shape, chunks):
    x = synthetic.input_batch(shape, 32) * 0.9 + 0.1
    mm, mn, mean, n = rangebn_stats((x if x.dim() == 4 else x[:, :, None, None]).to(gpu), chunks)
    wmm, wmn, wmean, wn = O.rangebn_chunk_stats(x, chunks)
    assert n == wn
    _close(mm, wmm)
    _close(mn, wmn)
    _close(mean, wmean)


def test_rangebn_stats_rejects_uneven_chunks(gpu):
    with pytest.raises(ValueError, match="num_chunks"):
        rangebn_stats(torch.zeros(3, 4, 5, 5, device=gpu), 16)


@pytest.mark.parametrize("name", ["c3x3_64_64_s1", "c7x7_3_64_s2", "fc_512_1000", "rbn_32", "c3x3_24_40_ragged"])
def test_layer_measure_mode_reproduces_reference_buffers(gpu, name):
    """The module path's measure mode (main.py:154-205) on the device, over the fixture's
    own calibration batches, against the reference-calibrated buffers."""
    d = load_fixture("layer_" + name)
    cfg = d["config"]
    kw = cfg["kw"]
    if cfg["kind"].startswith("conv"):
        mod = QConv2d(**kw, num_bits=8, num_bits_weight=8, num_bits_grad=8, biprecision=True)
    elif cfg["kind"] == "linear":
        mod = QLinear(**kw, num_bits=8, num_bits_weight=8, num_bits_grad=8, biprecision=True)
    else:
        mod = RangeBN(kw["num_features"], num_bits=8, num_bits_grad=8)
    wrap = nn.Sequential(mod)
    synthetic.init_params(wrap, seed=cfg["param_seed"])
    wrap = wrap.to(gpu)
    set_measure_mode(wrap, True)
    wrap.train()
    with torch.no_grad():
        for s in cfg["calib_seeds"]:
            wrap(synthetic.input_batch(tuple(cfg["shape"]), s, relu=cfg["relu_in"]).to(gpu))
    ref = fixture_buffers(d)
    for k, v in wrap.state_dict().items():
        if "running" in k or "num_measurements" in k:
            _close(v, ref[k])


def test_model_measure_mode_close_to_reference(gpu):
    """A whole model (ResNet-18 CIFAR fixture) calibrated on the device: every running
    statistic near the reference's (the float convs between layers run on different
    hardware, so the bar is looser than the per-kernel one)."""
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    for m in model.modules():  # start from fresh buffers, as the reference's calibration did
        if isinstance(m, RangeBN):
            m.running_mean.zero_()
            m.running_var.zero_()
        if hasattr(m, "num_measurements"):
            m.running_min.zero_(), m.running_max.zero_(), m.num_measurements.zero_()
            m.running_var.fill_(1.0), m.running_mean.zero_()
    cfg = d["config"]
    model = model.to(gpu)
    set_measure_mode(model, True)
    model.train()
    with torch.no_grad():
        for s in cfg["calib_seeds"]:
            model(synthetic.input_batch((cfg["calib_batch"],) + tuple(cfg["shape"][1:]), s).to(gpu))
    set_measure_mode(model, False)
    model.eval()
    for k, v in model.state_dict().items():
        if "running" in k or "num_measurements" in k:
            _close(v, ref[k], tol=1e-3)
