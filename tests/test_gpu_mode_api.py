"""The QuantNode mode API on the device (quantize.py:177-196, :547-610).

* overwrite_params bakes the fake-quantized weight and bias into the state_dict
  (QConv2d :301-312, QLinear :386-396): bit-exact against the oracle's uniform_quantize
  with the same tensor ranges;
* set_quant_mode(model, False) turns every QuantNode into the float layer
  (enable_quant False: F.conv2d / F.linear on the raw input, :350-352, :429-430);
* the frozen-range branch (freeze_param_dyn_range, :317-338): the stored weight/bias
  ranges feed the quantizers instead of fresh ones -- packed on the device and checked
  against the oracle at the per-layer bar.  (freeze_quant_params itself sets the
  misspelled attribute, :590, so it never reaches this branch: tests/test_mode_api.py.)
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import qnn_oracle as O
from qnn import synthetic
from qnn.quantize import QConv2d, QLinear, overwrite_params, set_quant_mode

pytestmark = pytest.mark.gpu

LAYER_TOL = 1e-5


def _net():
    net = nn.Sequential(QConv2d(8, 16, 3, padding=1, bias=True, num_bits_grad=8, biprecision=True),
                        QLinear(16, 10, bias=True, num_bits_grad=8, biprecision=True))
    synthetic.init_params(net, 11)
    for m in (net[0], net[1]):
        m.quantize_input.running_min.fill_(-1.5)
        m.quantize_input.running_max.fill_(2.25)
    return net.eval()


def _close(y, ref, tol=LAYER_TOL):
    y, ref = y.detach().float().cpu(), ref.detach().float().cpu()
    err = (y - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item() + 1e-6, err


def test_overwrite_params_bit_exact(gpu):
    net = _net().to(gpu)
    x = synthetic.input_batch((3, 8, 9, 9), 12).to(gpu)
    with torch.no_grad():
        net[0](x)  # a quantized forward refreshes weight_min/max and bias_min/max (:317-330)
        net[1](synthetic.input_batch((3, 16), 13).to(gpu))
    before = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    overwrite_params(net)
    after = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    for p in ("0.", "1."):
        wmin, wmax = before[p + "weight_min"], before[p + "weight_max"]
        want_w = O.uniform_quantize(before[p + "weight"], 8, wmin, wmax)
        want_b = O.uniform_quantize(before[p + "bias"], 8, before[p + "bias_min"], before[p + "bias_max"])
        assert torch.equal(after[p + "weight"], want_w), p + "weight"
        assert torch.equal(after[p + "bias"], want_b), p + "bias"
        # the range buffers are kept (load_state_dict of the updated dict)
        assert torch.equal(after[p + "weight_min"], wmin)


def test_set_quant_mode_false_is_the_float_layer(gpu):
    net = _net().to(gpu)
    x = synthetic.input_batch((2, 8, 7, 7), 14).to(gpu)
    set_quant_mode(net, False)
    assert not net[0].enable_quant and not net[0].quantize_input.enable_quant
    with torch.no_grad():
        y = net[0](x)
        ref = F.conv2d(x, net[0].weight, net[0].bias, 1, 1)
    assert torch.equal(y, ref)
    set_quant_mode(net, True)
    with torch.no_grad():
        yq = net[0](x)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    _close(yq, O.qconv2d(x.cpu(), sd["0.weight"], sd["0.bias"], 1, 1, 1, 1, (-1.5, 2.25)))


def test_frozen_range_pack_path(gpu):
    """freeze_param_dyn_range: the stored (narrower) weight and bias ranges are used, so the
    output differs from the fresh-range forward and matches the oracle's frozen branch."""
    net = _net()
    m = net[0]
    w = m.weight.detach()
    wmin = w.flatten(1).min(-1)[0].view(-1, 1, 1, 1) * 0.5  # clipped ranges: codes saturate
    wmax = w.flatten(1).max(-1)[0].view(-1, 1, 1, 1) * 0.5
    bmin, bmax = m.bias.detach().min() * 0.25, m.bias.detach().max() * 0.25
    with torch.no_grad():
        m.weight_min = wmin.clone()
        m.weight_max = wmax.clone()
        m.bias_min = bmin.clone()
        m.bias_max = bmax.clone()
    m.freeze_param_dyn_range = True
    net = net.to(gpu)
    x = synthetic.input_batch((2, 8, 9, 9), 15)
    with torch.no_grad():
        y = net[0](x.to(gpu))
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    ref = O.qconv2d(x, sd["0.weight"], sd["0.bias"], 1, 1, 1, 1, (-1.5, 2.25), frozen=(wmin, wmax, bmin, bmax))
    _close(y, ref)
    # the buffers were not refreshed (the frozen branch skips :317-330)
    assert torch.equal(net[0].weight_min.cpu(), wmin) and torch.equal(net[0].bias_max.cpu(), bmax)
    fresh = O.qconv2d(x, sd["0.weight"], sd["0.bias"], 1, 1, 1, 1, (-1.5, 2.25))
    assert (fresh - ref).abs().max().item() > 1e-3  # the frozen ranges really were used
