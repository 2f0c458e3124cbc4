"""Pin the oracle (oracle/qnn_oracle.py) to the reference's own outputs.

Fixtures in tests/golden/ were produced by the reference itself
(tools/gen_golden.py); the oracle must reproduce them BITWISE on CPU.  These
run without a GPU.
"""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_fixture
from fixtures_util import build_layer, build_model, oracle_layer
from oracle import qnn_oracle as O

LAYERS = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "layer_*.npz")))
MODELS = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "model_*.npz")))


def test_fixture_inventory():
    assert len(LAYERS) >= 15 and len(MODELS) >= 4


def test_quantize_kat_float_path():
    d = load_fixture("quantize_kat")
    n = 0
    while f"float/{n}/x" in d:
        x, (mn, mx), y = d[f"float/{n}/x"], d[f"float/{n}/range"], d[f"float/{n}/y"]
        got = O.uniform_quantize(torch.from_numpy(x), 8, float(mn), float(mx)).numpy()
        np.testing.assert_array_equal(got.view(np.uint32), y.view(np.uint32))
        # numpy restatement of the codes + dequantization is bitwise too
        q = O.quantize_codes_np(x, mn, mx)
        assert np.all((q >= 0) & (q <= 255)) and np.all(q == np.round(q))
        np.testing.assert_array_equal(O.dequantize_np(q, mn, mx), y)
        n += 1
    assert n >= 7


def test_quantize_kat_tensor_and_none_paths():
    d = load_fixture("quantize_kat")
    i = 0
    while f"tensor/{i}/x" in d:
        w = torch.from_numpy(d[f"tensor/{i}/x"])
        lo, hi = O.weight_ranges(w)
        got = O.uniform_quantize(w, 8, lo, hi).numpy()
        np.testing.assert_array_equal(got, d[f"tensor/{i}/y"])
        i += 1
    j = 0
    while f"none/{j}/x" in d:
        got = O.uniform_quantize(torch.from_numpy(d[f"none/{j}/x"]), 8).numpy()
        np.testing.assert_array_equal(got, d[f"none/{j}/y"])
        j += 1
    assert i >= 4 and j >= 3


@pytest.mark.parametrize("name", LAYERS)
def test_layer_fixture_bitwise(name):
    d = load_fixture("layer_" + name)
    wrap, _, x = build_layer(d)
    assert abs(float(x.double().abs().sum()) - float(d["x_checksum"])) <= 1e-9 * float(d["x_checksum"])
    y = oracle_layer(O, d, wrap, x)
    np.testing.assert_array_equal(y.numpy(), d["y"])


@pytest.mark.parametrize("name", MODELS)
def test_model_fixture_bitwise(name):
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    assert list(model.state_dict().keys()) == [str(k) for k in d["keys"]]
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    cfg = d["config"]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    logits = O.model_forward(sd, x, cfg["factory"], cfg["kw"])
    np.testing.assert_array_equal(logits.numpy(), d["logits"])
