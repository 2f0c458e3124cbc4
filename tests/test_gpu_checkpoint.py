"""Checkpoint loading on the device (qnn/checkpoint.py): a checkpoint
written from the golden fixture loads strictly, pre-packs every int8 operand at load
time, and reproduces the fixture model's logits bitwise (and the reference's golden
logits within the end-to-end bar); a checkpoint without calibrated buffers is calibrated
on the device over the fixture's calibration batches, writes the .measure checkpoint,
and the next load takes it."""
import pytest
import torch

from conftest import load_fixture
from fixtures_util import build_model, e2e_tolerance, oracle_fp64_drift
from oracle import qnn_oracle as O
from qnn import checkpoint as C
from qnn import synthetic
from qnn.quantize import QConv2d, QLinear
from qnn.resnet_quantized import resnet_quantized

pytestmark = pytest.mark.gpu


def _fresh():
    torch.manual_seed(0)
    return resnet_quantized(depth=18, dataset="cifar10").eval()


def test_checkpoint_prepacked_logits(gpu, tmp_path):
    d = load_fixture("model_resnet18_cifar")
    model, x = build_model(d)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    C.save_checkpoint(str(tmp_path / "ckpt.pth.tar"), model, "resnet", "{'depth': 18}", 91.0)
    fresh = _fresh()
    assert C.load_maybe_calibrate(fresh, str(tmp_path / "ckpt.pth.tar"), str(tmp_path), "resnet", 18,
                                  device=gpu) == "checkpoint"
    layers = [m for m in fresh.modules() if isinstance(m, (QConv2d, QLinear))]
    assert layers and all(m._qpack is not None for m in layers), "int8 operands not packed at load"
    keys = [m._qpack.key for m in layers]
    with torch.no_grad():
        y = fresh(x.to(gpu)).cpu()
        y_direct = model.to(gpu)(x.to(gpu)).cpu()
    assert [m._qpack.key for m in layers] == keys, "the first forward re-packed"
    assert torch.equal(y, y_direct)
    ref = torch.from_numpy(d["logits"])
    drift64, _ = oracle_fp64_drift(O, sd, x, d["config"]["factory"], d["config"]["kw"], ref)
    assert (y - ref).abs().max().item() <= e2e_tolerance(ref, drift64)


def test_calibrate_then_measure_file(gpu, tmp_path):
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    ref = model.state_dict()
    bare = {k: v for k, v in ref.items() if "quantize_input" not in k and "running" not in k}
    cfg = d["config"]
    batches = [synthetic.input_batch((cfg["calib_batch"],) + tuple(cfg["shape"][1:]), s) for s in cfg["calib_seeds"]]
    fresh = _fresh()
    for m in fresh.modules():  # a float checkpoint's model starts from fresh statistics
        if hasattr(m, "num_measurements"):
            m.running_min.zero_(), m.running_max.zero_(), m.num_measurements.zero_()
            m.running_var.fill_(1.0), m.running_mean.zero_()
        elif hasattr(m, "running_mean"):
            m.running_mean.zero_(), m.running_var.zero_()
    assert C.load_maybe_calibrate(fresh, bare, str(tmp_path), "resnet", 18, calib_batches=batches,
                                  device=gpu) == "calibrated"
    mpath = tmp_path / C.measure_name("resnet", 18)
    msd, meta = C.load_checkpoint(mpath)
    assert set(meta) == {"epoch", "model", "config", "best_prec1", "regime"}
    for k, v in fresh.state_dict().items():
        if "running" in k:
            r = ref[k]
            assert bool(((v.cpu() - r).abs() <= 1e-3 * r.abs().clamp_min(1.0)).all()), k
    again = _fresh()
    # pack=False: packing refreshes weight_min/max from the weights, as the reference's first
    # eval forward does (quantize.py:316-330); the loaded state itself must equal the file
    assert C.load_maybe_calibrate(again, bare, str(tmp_path), "resnet", 18, device=gpu, pack=False) == "measure"
    assert all(torch.equal(v.cpu(), msd[k]) for k, v in again.state_dict().items())
    assert C.prepack(again) > 0
