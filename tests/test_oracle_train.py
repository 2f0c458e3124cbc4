"""The oracle's training-side restatement pinned to the reference.

tests/golden/train_*.npz hold one reference QConv2d / QLinear in training mode
(tools/gen_golden.py gen_train): forward on a fresh batch (QuantMeasure batch statistics),
backward of a fixed output gradient, with the gradient quantizer's stochastic-rounding draw
recorded.  oracle.qlayer_train with that draw must reproduce the output and every gradient
BITWISE (same CPU ops in the same order: straight-through quantizers, UniformQuantizeGrad's
enforce_true_zero branch, the biprecision split)."""
import glob
import os

import pytest
import torch

from conftest import GOLDEN, load_fixture
from oracle import qnn_oracle as O
from qnn import synthetic
from qnn.quantize import QConv2d, QLinear

TRAIN = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "train_*.npz")))


def train_params(d):
    """The fixture layer's parameters, rebuilt with the generator's initializer."""
    cfg = d["config"]
    torch.manual_seed(0)
    args = dict(num_bits=8, num_bits_weight=8, num_bits_grad=cfg["num_bits_grad"], biprecision=cfg["biprecision"])
    mod = QConv2d(**cfg["kw"], **args) if cfg["kind"] == "conv" else QLinear(**cfg["kw"], **args)
    wrap = torch.nn.Sequential(mod)
    synthetic.init_params(wrap, seed=cfg["param_seed"])
    assert abs(synthetic.param_checksum(wrap) - float(d["param_checksum"])) <= 1e-9 * abs(float(d["param_checksum"]))
    return mod


def oracle_train(d, x, w, b, xrange):
    cfg = d["config"]
    conv = None
    if cfg["kind"] == "conv":
        kw = cfg["kw"]
        conv = (kw.get("stride", 1), kw.get("padding", 0), 1, 1)
    noise = torch.from_numpy(d["noise"]) if cfg["num_bits_grad"] is not None else None
    return O.qlayer_train(x, w, b, xrange, conv=conv, num_bits_grad=cfg["num_bits_grad"],
                          biprecision=cfg["biprecision"], noise=noise)


def test_train_fixtures_present():
    assert len(TRAIN) >= 4


@pytest.mark.parametrize("name", TRAIN)
def test_oracle_train_bitwise_vs_reference(name):
    d = load_fixture(name)
    mod = train_params(d)
    x = torch.from_numpy(d["x"]).requires_grad_(True)
    w = mod.weight.detach().clone().requires_grad_(True)
    b = None if mod.bias is None else mod.bias.detach().clone().requires_grad_(True)
    mn, mx, _, _ = O.measure_stats(x)
    y = oracle_train(d, x, w, b, (float(mn), float(mx)))
    assert torch.equal(y.detach(), torch.from_numpy(d["y"]))
    y.backward(torch.from_numpy(d["gy"]))
    assert torch.equal(x.grad, torch.from_numpy(d["grad_x"]))
    assert torch.equal(w.grad, torch.from_numpy(d["grad_w"]))
    if b is not None:
        assert torch.equal(b.grad, torch.from_numpy(d["grad_b"]))
