"""The oracle's calibration restatement (oracle.calibrate_*) against the
reference-calibrated buffers of every layer fixture (tools/gen_golden.py ran the
reference's measure mode, main.py:154-205, on the calibration batches rebuilt here from
their seeds): QuantMeasure train statistics (quantize.py:216-236) and RangeBN's chunked
mean / scale (:466-482) reproduce bitwise."""

import numpy as np
import pytest
import torch

from conftest import load_fixture
from oracle import qnn_oracle as O
from qnn import synthetic

LAYERS = ["c3x3_64_64_s1", "c3x3_64_128_s2", "c1x1_256_64", "c1x1_64_128_s2", "c7x7_3_64_s2", "c3x3_3_32_s2",
          "dw3x3_32_s1_bias", "dw3x3_64_s2_bias", "c3x3_16_16_cifar", "c3x3_512_512_k4608", "c3x3_24_40_ragged",
          "c3x3_64_64_aciq", "fc_512_1000", "fc_64_10", "rbn_32"]


def _calib_batches(cfg):
    return [synthetic.input_batch(tuple(cfg["shape"]), s, relu=cfg["relu_in"]) for s in cfg["calib_seeds"]]


@pytest.mark.parametrize("name", LAYERS)
def test_measure_stats_bitwise_vs_reference(name):
    d = load_fixture("layer_" + name)
    cfg = d["config"]
    st = O.measure_state()
    for x in _calib_batches(cfg):
        O.calibrate_measure(st, x)
    for k, v in st.items():
        ref = d[f"buf/0.quantize_input.{k}"]
        assert np.array_equal(v.numpy(), ref), (k, v.numpy(), ref)


def test_rangebn_stats_bitwise_vs_reference():
    d = load_fixture("layer_rbn_32")
    cfg = d["config"]
    st = {"running_mean": torch.zeros(cfg["kw"]["num_features"]), "running_var": torch.zeros(cfg["kw"]["num_features"]),
          "measure": O.measure_state()}
    for x in _calib_batches(cfg):
        O.calibrate_rangebn(st, x)
    assert np.array_equal(st["running_mean"].numpy(), d["buf/0.running_mean"])
    assert np.array_equal(st["running_var"].numpy(), d["buf/0.running_var"])
    for k, v in st["measure"].items():
        assert np.array_equal(v.numpy(), d[f"buf/0.quantize_input.{k}"]), k


def test_momentum_rule_is_a_running_average():
    """num_measurements / (num_measurements + 1): after n batches the running stat is the
    plain mean of the n batch statistics (quantize.py:216-219)."""
    st = O.measure_state()
    xs = [synthetic.input_batch((3, 4, 5, 5), 900 + i) for i in range(4)]
    mins = [O.calibrate_measure(st, x)[0].item() for x in xs]
    assert st["running_min"].item() == pytest.approx(float(np.mean(mins)), rel=1e-6)
    assert st["num_measurements"].item() == 4
