"""The QuantNode tree helpers on CPU (no compute): quantize.py:177-196, :547-610.

set_measure_mode flips enable_quant on every QuantNode (QConv2d, QLinear and their
QuantMeasure children) and puts BatchNorm into eval for measure=True (:547-558);
set_quant_mode sets enable_quant (:561-568); freeze_quant_params switches every
QuantMeasure to eval (train(not freeze)), optionally changes its momentum, and sets the
MISSPELLED attribute `freeze_param_dyn_rang` (:579-592) -- so freeze_param_dyn_range, the
flag QConv2d.forward reads (:317), stays False; set_global_quantization_method sets the
QuantMeasure method (:602-610).
"""
import torch.nn as nn

from qnn.quantize import (QConv2d, QLinear, QuantMeasure, RangeBN, freeze_quant_params, set_global_quantization_method,
                          set_measure_mode, set_quant_mode)


def _net():
    return nn.Sequential(QConv2d(4, 8, 3, padding=1), nn.BatchNorm2d(8), RangeBN(8), nn.Flatten(), QLinear(8, 3))


def _qnodes(net):
    return [m for m in net.modules() if isinstance(m, (QConv2d, QLinear, QuantMeasure))]


def test_set_measure_mode():
    net = _net().train()
    set_measure_mode(net, True)
    assert not net[1].training  # BatchNorm -> eval while measuring
    assert all(not m.enable_quant for m in _qnodes(net))
    # RangeBN is neither BN nor a QuantNode: it stays in train mode, while
    # recursive_apply still reaches its QuantMeasure child
    assert net[2].training and not net[2].quantize_input.enable_quant
    set_measure_mode(net, False)
    assert net[1].training and all(m.enable_quant for m in _qnodes(net))


def test_set_measure_mode_momentum_reaches_quantmeasure():
    net = _net()
    set_measure_mode(net, True, momentum=0.3)
    assert net[0].quantize_input.momentum == 0.3 and net[4].quantize_input.momentum == 0.3


def test_set_quant_mode():
    net = _net()
    set_quant_mode(net, False)
    assert all(not m.enable_quant for m in _qnodes(net))
    set_quant_mode(net, True)
    assert all(m.enable_quant for m in _qnodes(net))


def test_freeze_quant_params_typo_kept():
    net = _net().train()
    freeze_quant_params(net, freeze=True, momentum=0.05)
    for m in net.modules():
        if isinstance(m, QuantMeasure):
            assert not m.training and m.momentum == 0.05
    for m in (net[0], net[4]):
        assert m.freeze_param_dyn_rang is True  # (sic) quantize.py:590
        assert m.freeze_param_dyn_range is False  # so the weight range is never frozen
    freeze_quant_params(net, freeze=False)
    assert all(m.training for m in net.modules() if isinstance(m, QuantMeasure))
    assert net[0].quantize_input.momentum == 0.05  # momentum='same' keeps it


def test_set_global_quantization_method():
    net = _net()
    set_global_quantization_method(net, "aciq")
    assert all(m.method == "aciq" for m in net.modules() if isinstance(m, QuantMeasure))
    set_global_quantization_method(net, "avg")
    assert all(m.method == "avg" for m in net.modules() if isinstance(m, QuantMeasure))
