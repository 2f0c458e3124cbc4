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
    """Largest max|logit - ref| of the oracle (== the reference, bitwise) over two
    equally valid re-orderings of its contraction: (a) fp64 accumulation, (b) fp32
    split-K (input channels summed in two halves).  This is the reference's own
    sensitivity to accumulation order, which requantization flips amplify
    (SURVEY.md §0.6); end-to-end tolerances scale with it."""
    import torch.nn.functional as F
    c2, l2 = F.conv2d, F.linear

    def conv64(a, w, b=None, *r):
        return c2(a.double(), w.double(), None if b is None else b.double(), *r).float()

    def lin64(a, w, b=None):
        return l2(a.double(), w.double(), None if b is None else b.double()).float()

    def conv_split(a, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        if groups != 1 or a.shape[1] < 2:
            return c2(a, w, b, stride, padding, dilation, groups)
        h = a.shape[1] // 2
        y = c2(a[:, :h], w[:, :h], None, stride, padding, dilation) + c2(a[:, h:], w[:, h:], None, stride, padding,
                                                                           dilation)
        return y if b is None else y + b.view(1, -1, 1, 1)

    def lin_split(a, w, b=None):
        h = a.shape[1] // 2
        y = l2(a[:, :h], w[:, :h]) + l2(a[:, h:], w[:, h:])
        return y if b is None else y + b

    worst, y_worst = -1.0, None
    for cv, ln in ((conv64, lin64), (conv_split, lin_split)):
        try:
            oracle.F.conv2d, oracle.F.linear = cv, ln
            y = oracle.model_forward({k: v.clone() for k, v in sd.items()}, x, factory, kw)
        finally:
            oracle.F.conv2d, oracle.F.linear = c2, l2
        dev = (y - ref).abs().max().item()
        if dev > worst:
            worst, y_worst = dev, y
    return worst, y_worst


def e2e_tolerance(ref, drift64):
    return max(3e-2 * ref.abs().max().item(), 1.5 * drift64)
