"""Rebuild golden-fixture layers/models with this package's modules (CPU construction)."""
import torch
import torch.nn as nn

from conftest import fixture_buffers
from qnn import synthetic
from qnn.mobilenet_quantized import mobilenet_quantized
from qnn.quantize import QConv2d, QLinear, RangeBN, set_global_quantization_method
from qnn.resnet_quantized import resnet_quantized

BIPREC = dict(num_bits=8, num_bits_weight=8, num_bits_grad=8, biprecision=True)


def build_layer(d):
    """-> (wrapper Sequential, module, eval input x) exactly as tools/gen_golden.py built them."""
    cfg = d["config"]
    kind, kw = cfg["kind"], cfg["kw"]
    torch.manual_seed(0)
    if kind in ("conv", "conv_aciq"):
        m = QConv2d(**kw, **BIPREC)
    elif kind == "linear":
        m = QLinear(**kw, **BIPREC)
    else:
        m = RangeBN(kw["num_features"], num_bits=8, num_bits_grad=8)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, cfg["param_seed"])
    assert abs(synthetic.param_checksum(wrap) - float(d["param_checksum"])) <= 1e-9 * float(d["param_checksum"])
    sd = wrap.state_dict()
    sd.update(fixture_buffers(d))
    wrap.load_state_dict(sd, strict=True)
    wrap.eval()
    if kind == "conv_aciq":
        set_global_quantization_method(wrap, "aciq")
    x = synthetic.input_batch(cfg["shape"], cfg["eval_seed"], relu=cfg["relu_in"]) * cfg["eval_scale"]
    return wrap, m, x


def build_model(d):
    cfg = d["config"]
    torch.manual_seed(0)
    if cfg["factory"] == "resnet":
        model = resnet_quantized(**cfg["kw"])
    else:
        model = mobilenet_quantized(**cfg["kw"])
    synthetic.init_params(model, cfg["param_seed"])
    assert abs(synthetic.param_checksum(model) - float(d["param_checksum"])) <= 1e-9 * float(d["param_checksum"])
    sd = model.state_dict()
    sd.update(fixture_buffers(d))
    model.load_state_dict(sd, strict=True)
    model.eval()
    x = synthetic.input_batch(cfg["shape"], cfg["eval_seed"])
    return model, x


def oracle_layer(oracle, d, wrap, x):
    """Oracle output of a fixture layer on input x (CPU)."""
    cfg = d["config"]
    sd = {k: v.clone() for k, v in wrap.state_dict().items()}
    method = "aciq" if cfg["kind"] == "conv_aciq" else "avg"
    rng = oracle.measure_range(sd, "0.quantize_input.", method)
    if cfg["kind"].startswith("conv"):
        kw = cfg["kw"]
        return oracle.qconv2d(x, sd["0.weight"], sd.get("0.bias"), kw.get("stride", 1), kw.get("padding", 0), 1,
                              kw.get("groups", 1), rng)
    if cfg["kind"] == "linear":
        return oracle.qlinear(x, sd["0.weight"], sd.get("0.bias"), rng)
    return oracle.rangebn(x, sd["0.running_mean"], sd["0.running_var"], sd["0.weight"], sd["0.bias"], rng)


def oracle_fp64_drift(oracle, sd, x, factory, kw, ref):
    """max|logit - ref| of the oracle (== the reference, bitwise) when its contraction
    runs in fp64: the reference's own sensitivity to accumulation order, which
    requantization flips amplify.  End-to-end tolerances scale with it."""
    import torch.nn.functional as F
    c2, l2 = F.conv2d, F.linear
    try:
        oracle.F.conv2d = lambda a, w, b=None, *r: c2(a.double(), w.double(), None if b is None else b.double(), *r).float()
        oracle.F.linear = lambda a, w, b=None: l2(a.double(), w.double(), None if b is None else b.double()).float()
        y64 = oracle.model_forward({k: v.clone() for k, v in sd.items()}, x, factory, kw)
    finally:
        oracle.F.conv2d, oracle.F.linear = c2, l2
    return (y64 - ref).abs().max().item(), y64


def e2e_tolerance(ref, drift64):
    return max(3e-2 * ref.abs().max().item(), 1.5 * drift64)
