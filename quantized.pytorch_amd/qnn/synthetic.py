"""Deterministic synthetic parameters and inputs (numpy PCG64, torch-RNG free).

The reference initialises with torch's RNG (`models/resnet_quantized.py:19-34`,
`models/mobilenet_quantized.py:20-30`).  Golden fixtures and the benchmark need
weights that both the reference import (fixture generation) and this package
(tests, bench) can rebuild bit-for-bit without shipping state_dicts, so every
tensor here is drawn from `numpy.random.Generator(PCG64(SeedSequence([seed, i])))`
in state_dict order.  Laws:

* QConv2d weight  ~ N(0, sqrt(2 / (kh*kw*Cout)))  (the reference init law, :22-23)
* QConv2d bias    ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in))  (nn.Conv2d default law)
* RangeBN weight  ~ U(0.5, 1.5), bias ~ U(-0.1, 0.1)   (stated deviation from
  the reference's w=1/b=0 and zero-init last BN, which make quantizers degenerate)
* QLinear weight  ~ N(0, 0.01), bias ~ U(-0.01, 0.01)   (reference zeroes the bias)
* inputs          ~ N(0, 1) float32 (ImageNet-normalised statistics, data.py:26)
"""
import math

import numpy as np
import torch


def _gen(seed, idx):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([int(seed), int(idx)])))


def normal(shape, seed, idx=0, std=1.0):
    g = _gen(seed, idx)
    a = g.standard_normal(size=tuple(shape), dtype=np.float32)
    if std != 1.0:
        a = (a * np.float32(std)).astype(np.float32)
    return a


def uniform(shape, lo, hi, seed, idx=0):
    g = _gen(seed, idx)
    a = g.random(size=tuple(shape), dtype=np.float32)
    return (np.float32(lo) + a * np.float32(hi - lo)).astype(np.float32)


def input_batch(shape, seed, relu=False):
    a = normal(shape, seed, 0)
    if relu:
        a = np.maximum(a, np.float32(0))
    return torch.from_numpy(a)


def init_params(model, seed):
    """Overwrite every QConv2d / QLinear / RangeBN parameter of `model` in place.

    Works on the reference modules and on this package's modules alike (it keys
    on class names), so both sides build identical weights from one seed.
    """
    idx = 0
    with torch.no_grad():
        for name, m in model.named_modules():
            kind = type(m).__name__
            if kind == "QConv2d":
                kh, kw = m.kernel_size
                w = normal(m.weight.shape, seed, idx, math.sqrt(2.0 / (kh * kw * m.out_channels)))
                m.weight.copy_(torch.from_numpy(w)); idx += 1
                if m.bias is not None:
                    fan_in = (m.in_channels // m.groups) * kh * kw
                    b = 1.0 / math.sqrt(fan_in)
                    m.bias.copy_(torch.from_numpy(uniform(m.bias.shape, -b, b, seed, idx))); idx += 1
            elif kind == "QLinear":
                m.weight.copy_(torch.from_numpy(normal(m.weight.shape, seed, idx, 0.01))); idx += 1
                if m.bias is not None:
                    m.bias.copy_(torch.from_numpy(uniform(m.bias.shape, -0.01, 0.01, seed, idx))); idx += 1
            elif kind == "RangeBN":
                m.weight.copy_(torch.from_numpy(uniform(m.weight.shape, 0.5, 1.5, seed, idx))); idx += 1
                m.bias.copy_(torch.from_numpy(uniform(m.bias.shape, -0.1, 0.1, seed, idx))); idx += 1
    return model


def param_checksum(model):
    """float64 sum of |param| over all parameters: cheap drift detector for fixtures."""
    return float(sum(p.detach().double().abs().sum().item() for p in model.parameters()))
