"""Checkpoint loading (qnn/checkpoint.py; main.py:154-205) on the CPU:
the {'state_dict', ...} wrapper and bare state_dicts, weights-only loading (a file that
needs code to unpickle is refused), and the three outcomes of load_maybe_calibrate.
The checkpoint files are written by the test from the golden fixtures (the reference's
calibrated buffers), not by the loader under test."""
import collections

import pytest
import torch

from conftest import load_fixture
from fixtures_util import build_model
from qnn import checkpoint as C
from qnn.resnet_quantized import resnet_quantized


class NotATensor:  # a pickled instance of this needs code from this module to load
    def __init__(self):
        self.x = 1


def _fixture_model():
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    return model, d


def _fresh():
    torch.manual_seed(0)
    return resnet_quantized(depth=18, dataset="cifar10").eval()


def _write(path, sd, wrap=True):
    obj = {"epoch": 0, "model": "resnet", "config": "{'depth': 18}", "state_dict": sd, "best_prec1": 91.25,
           "regime": [{"epoch": 0, "optimizer": "SGD", "lr": 0.1}]} if wrap else sd
    torch.save(obj, path)


def test_wrapper_and_bare_state_dict(tmp_path):
    model, _ = _fixture_model()
    sd = model.state_dict()
    _write(tmp_path / "a.pth.tar", sd)
    _write(tmp_path / "b.pth", collections.OrderedDict(sd), wrap=False)
    sa, meta = C.load_checkpoint(tmp_path / "a.pth.tar")
    sb, meta_b = C.load_checkpoint(tmp_path / "b.pth")
    assert meta["best_prec1"] == 91.25 and meta["regime"][0]["optimizer"] == "SGD" and meta_b == {}
    assert list(sa) == list(sd) == list(sb)
    assert all(torch.equal(sa[k], sd[k]) and torch.equal(sb[k], sd[k]) for k in sd)


def test_code_carrying_pickle_is_refused(tmp_path):
    torch.save({"state_dict": {}, "extra": NotATensor()}, tmp_path / "evil.pth")
    with pytest.raises(Exception, match="(?i)weights.only|unpickl|global"):
        C.load_checkpoint(tmp_path / "evil.pth")


def test_strict_checkpoint_loads_every_buffer(tmp_path):
    model, _ = _fixture_model()
    _write(tmp_path / "ckpt.pth.tar", model.state_dict())
    fresh = _fresh()
    how = C.load_maybe_calibrate(fresh, str(tmp_path / "ckpt.pth.tar"), str(tmp_path), "resnet", 18, pack=False)
    assert how == "checkpoint"
    ref = model.state_dict()
    assert all(torch.equal(v, ref[k]) for k, v in fresh.state_dict().items())


def _uncalibrated(sd):
    return {k: v for k, v in sd.items() if "quantize_input" not in k and "running" not in k}


def test_measure_file_is_used_when_buffers_are_missing(tmp_path):
    model, _ = _fixture_model()
    C.save_checkpoint(str(tmp_path / C.measure_name("resnet", 18)), model, "resnet", "{'depth': 18}", 90.0)
    fresh = _fresh()
    how = C.load_maybe_calibrate(fresh, _uncalibrated(model.state_dict()), str(tmp_path), "resnet", 18, pack=False)
    assert how == "measure"
    ref = model.state_dict()
    assert all(torch.equal(v, ref[k]) for k, v in fresh.state_dict().items())


def test_missing_buffers_without_measure_or_data_is_an_error(tmp_path):
    model, _ = _fixture_model()
    with pytest.raises(RuntimeError, match="calib_batches"):
        C.load_maybe_calibrate(_fresh(), _uncalibrated(model.state_dict()), str(tmp_path), "resnet", 18, pack=False)
