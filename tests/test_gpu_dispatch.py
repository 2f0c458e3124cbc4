"""The reference's own forward (`output = model(inputs)`, main.py:359) on the fused engine
(qnn/dispatch.py): a plain eval forward of ResNet / MobileNet runs a cached qnn.Engine whose
logits are BITWISE the per-module path's; hooks, train mode, autograd, the 'aciq' method and a
new batch shape fall back to the module path (a new shape builds its own engine when it repeats).
"""
import pytest
import torch

from conftest import load_fixture
from fixtures_util import build_model
from qnn import dispatch as D
from qnn import synthetic
from qnn.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.fixture
def policy():
    old = D.DISPATCH[0]
    yield D.DISPATCH
    D.DISPATCH[0] = old


class _Count:
    """Counts engine replays (Engine.__call__) while active."""

    def __init__(self, monkeypatch):
        self.n = 0
        orig = Engine.__call__

        def wrapped(eng, x=None):
            self.n += 1
            return orig(eng, x)

        monkeypatch.setattr(Engine, "__call__", wrapped)


def _module_path(model, x, policy):
    policy[0] = "off"
    with torch.no_grad():
        y = model(x).clone()
    return y


@pytest.mark.parametrize("fixture,batch", [("model_resnet18_imagenet", 6), ("model_resnet18_cifar", 5),
                                           ("model_mobilenet", 3), ("model_resnet50_imagenet", 4)])
def test_dispatch_bitwise_module_path(gpu, policy, monkeypatch, fixture, batch):
    d = load_fixture(fixture)
    model, _ = build_model(d)
    model = model.to(gpu)
    x = synthetic.input_batch((batch,) + tuple(d["config"]["shape"][1:]), 31).to(gpu)
    ref = _module_path(model, x, policy)
    count = _Count(monkeypatch)
    policy[0] = "auto"
    outs = []
    with torch.no_grad():
        for _ in range(4):
            outs.append(model(x))
    eng = D.engine_for(model, x.shape)
    assert eng is not None, model.__dict__["_qnn_dispatch"].failed
    assert count.n >= 2, "the repeated eval forward did not reach the engine"
    for y in outs:
        assert torch.equal(y, ref), "dispatched logits != the per-module path"
    # a fresh tensor per call (the engine's static logits are not handed out)
    assert outs[-1].data_ptr() != outs[-2].data_ptr() and outs[-1].data_ptr() != eng.logits.data_ptr()


def test_dispatch_fallbacks(gpu, policy, monkeypatch):
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    model = model.to(gpu)
    x = synthetic.input_batch((4, 3, 32, 32), 32).to(gpu)
    ref = _module_path(model, x, policy)
    count = _Count(monkeypatch)
    policy[0] = "eager"
    with torch.no_grad():
        assert torch.equal(model(x), ref)
    assert count.n == 1
    # a forward hook: the module path (the hook sees the per-module tensors)
    seen = []
    h = model.layer1.register_forward_hook(lambda m, i, o: seen.append(o.shape))
    with torch.no_grad():
        assert torch.equal(model(x), ref)
    h.remove()
    assert count.n == 1 and seen == [torch.Size([4, 16, 32, 32])]
    # autograd on (parameters require grad): the module path, differentiable
    y = model(x)
    assert y.requires_grad and count.n == 1
    assert torch.equal(y.detach(), ref)
    # a new batch shape gets its own engine; the first shape's stays cached
    x2 = synthetic.input_batch((3, 3, 32, 32), 33).to(gpu)
    ref2 = _module_path(model, x2, policy)
    policy[0] = "auto"
    with torch.no_grad():
        y2a = model(x2)  # first sight: module path
        assert count.n == 1 and D.engine_for(model, x2.shape) is None
        y2b = model(x2)  # repeated: engine
        assert count.n == 2 and D.engine_for(model, x2.shape) is not None
        assert torch.equal(model(x), ref)  # the first shape's engine, still cached
    assert count.n == 3
    assert torch.equal(y2a, ref2) and torch.equal(y2b, ref2)
    # changed weights: a new engine with the new weights (the previous tile choice reused)
    old = D.engine_for(model, x.shape)
    with torch.no_grad():
        model.fc.weight.mul_(0.5)
    ref3 = _module_path(model, x, policy)
    policy[0] = "eager"
    with torch.no_grad():
        y3 = model(x)
    assert D.engine_for(model, x.shape) is not old
    assert torch.equal(y3, ref3) and not torch.equal(y3, ref)
    # the 'aciq' range method mutates running_var on every forward: the module path
    from qnn.quantize import set_global_quantization_method
    set_global_quantization_method(model, "aciq")
    n0 = count.n
    with torch.no_grad():
        model(x)
    assert count.n == n0
    set_global_quantization_method(model, "avg")
    # train mode (calibration): the module path, whose statistics update
    model.train()
    nm = model.conv1.quantize_input.num_measurements.clone()
    with torch.no_grad():
        model(x)
    assert count.n == n0 and model.conv1.quantize_input.num_measurements.item() == nm.item() + 1
