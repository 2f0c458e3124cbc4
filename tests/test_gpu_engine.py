"""Fused whole-network engine (qnn/engine.py) on the GPU.

* The engine evaluates the same contraction and restates the same elementwise
  chain (RangeBN eval -> residual -> ReLU -> requantize, code-domain max-pool,
  fused depthwise) as the module path, so the feature map entering the
  classifier head must be BITWISE equal to the module path's — whose every layer
  is checked against the oracle in tests/test_gpu_parity.py.
* Logits: the drift-calibrated end-to-end bar against the reference's golden
  logits (tests/test_gpu_parity.py docstring), and BITWISE the module path's (the
  engine's avg-pool sums in torch's AvgPool2d order, graph.hip avgpool_quant_kernel).
* Graph replay is deterministic and batch-size independent per sample.
"""
import glob
import os

import pytest
import torch

from conftest import GOLDEN, load_fixture
from fixtures_util import build_model, e2e_tolerance, oracle_fp64_drift
from oracle import qnn_oracle as O
from qnn.engine import Engine

pytestmark = pytest.mark.gpu
MODELS = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "model_*.npz")))


def _module_path(model, x):
    feats = {}
    pool = model.avg_pool if hasattr(model, "avg_pool") else model.avgpool
    def grab(m, i, o):  # a hook must return None (a returned value replaces the output)
        feats["x"] = i[0].detach().clone()

    h = pool.register_forward_hook(grab)
    with torch.no_grad():
        logits = model(x)
    h.remove()
    return logits, feats["x"]


@pytest.mark.parametrize("name", MODELS)
def test_engine_matches_module_path_and_reference(gpu, name):
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    ref = torch.from_numpy(d["logits"])
    model = model.to(gpu)
    xg = x.to(gpu)
    mod_logits, mod_feat = _module_path(model, xg)
    eng = Engine(model, batch=x.shape[0])
    logits = eng(xg).clone()
    # bitwise: every fused epilogue, the code-domain max-pool and the fused depthwise
    assert torch.equal(eng.head_input, mod_feat.permute(0, 2, 3, 1)), "engine feature map != module path"
    # bitwise the module path's logits (avg-pool in torch's summation order)
    assert torch.equal(logits, mod_logits), (logits - mod_logits).abs().max().item()
    # end-to-end vs the reference
    drift, _ = oracle_fp64_drift(O, sd, x, d["config"]["factory"], d["config"]["kw"], ref)
    err = (logits.cpu() - ref).abs().max().item()
    assert err <= e2e_tolerance(ref, drift), (err, drift)
    # graph replay is deterministic
    again = eng(xg).clone()
    assert torch.equal(again, logits)


def test_engine_batch_independence(gpu):
    """Per-sample results do not depend on the batch they run in (the DP sharding
    contract): batch 4 == 2 x batch 2, bitwise."""
    d = load_fixture("model_resnet18_cifar")
    model, _ = build_model(d)
    model = model.to(gpu)
    from qnn import synthetic
    x = synthetic.input_batch((4, 3, 32, 32), 77).to(gpu)
    full = Engine(model, batch=4)(x).clone()
    half = Engine(model, batch=2)
    a = half(x[:2]).clone()
    b = half(x[2:]).clone()
    assert torch.equal(full, torch.cat([a, b]))


def test_engine_launch_count_resnet18(gpu):
    from qnn import synthetic
    from qnn.resnet_quantized import resnet_quantized
    m = resnet_quantized(depth=18, dataset="imagenet")
    synthetic.init_params(m, 1)
    for mod in m.modules():
        if hasattr(mod, "running_min"):
            mod.running_min.fill_(0.0)
            mod.running_max.fill_(2.0)
        if type(mod).__name__ == "RangeBN":
            mod.running_var.fill_(0.5)
    m = m.to(gpu).eval()
    eng = Engine(m, batch=2, graph=False)
    # s2d quantize + the fused stem conv/max-pool (qnn_qconv2d_maxpool_fwd) + 19 block convs
    # (incl. 3 downsample) + avgpool + fc
    assert eng.num_launches == 1 + 1 + 19 + 1 + 1
    assert eng.launch_names.count("qnn_qconv2d_maxpool_fwd") == 1
    y = eng()
    assert torch.isfinite(y).all()


@pytest.mark.parametrize("max_links", [0, 1, 2, 3])
@pytest.mark.parametrize("name", ["resnet18_imagenet", "resnet50_imagenet"])
def test_engine_chain_length_bitwise(gpu, name, max_links):
    """Every residual chain limit (0 = an fp32 map at every identity shortcut) gives the
    same feature map entering the head as the module path, bitwise: the chain links
    recompute the fp32 block inputs with their producers' exact ops."""
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    model = model.to(gpu)
    xg = x.to(gpu)
    _, mod_feat = _module_path(model, xg)
    eng = Engine(model, batch=x.shape[0], max_links=max_links)
    eng(xg)
    assert torch.equal(eng.head_input, mod_feat.permute(0, 2, 3, 1)), f"max_links={max_links}: != module path"


@pytest.mark.parametrize("max_links", [0, 2, 4])
@pytest.mark.parametrize("name", ["resnet18_imagenet", "resnet50_imagenet", "resnet18_cifar"])
def test_engine_split_chain_bitwise(gpu, name, max_links):
    """The residual-chain tail of every block's last conv as its own launch
    (qnn_chain_epilogue, Engine(split_chain=True)) gives the same head input and logits as
    the fused general epilogue, bitwise, at every chain length (fp32 checkpoints, links)."""
    d = load_fixture("model_" + name)
    model, x = build_model(d)
    model = model.to(gpu)
    xg = x.to(gpu)
    fused = Engine(model, batch=x.shape[0], max_links=max_links, split_chain=False, autotune=False)
    yf = fused(xg).clone()
    hf = fused.head_input.clone()
    split = Engine(model, batch=x.shape[0], max_links=max_links, split_chain=True, autotune=False)
    assert split.launch_names.count("qnn_chain_epilogue") == len(Engine._blocks(model))
    ys = split(xg)
    assert torch.equal(split.head_input, hf)
    assert torch.equal(ys, yf)
