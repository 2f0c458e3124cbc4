"""Training-side quantization on the GPU, against the oracle's restatement,
which tests/test_oracle_train.py pins bitwise to the reference.

* The gradient quantizer (qnn_grad_quant_f32: UniformQuantizeGrad's enforce_true_zero branch
  with the stochastic-rounding draw given) is elementwise fp32 in the reference's op order:
  BITWISE equal to oracle.grad_quantize on the same gradient and draw.
* QConv2d / QLinear in train mode with autograd: the forward is the int8 kernel (per-layer bar
  against the oracle at the range the device measured); the backward restates the reference's
  straight-through / num_bits_grad / biprecision graph with fp32 transposed contractions, so the
  gradients match the oracle's within fp32 summation order: max|d| <= 1e-4 * max|ref|.
  The gradient quantizer is fed the fixture's recorded draw (qnn.quantize.GRAD_NOISE)."""
import pytest
import torch

from conftest import load_fixture
from oracle import qnn_oracle as O
from qnn import quantize as Q
from test_oracle_train import TRAIN, oracle_train, train_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stochastic", [False, True])
@pytest.mark.parametrize("shape", [(4, 32, 9, 9), (1000,), (3, 7)])
def test_grad_quantizer_bitwise(gpu, shape, stochastic):
    g = torch.randn(shape, generator=torch.Generator().manual_seed(5)) * 1e-3
    noise = torch.empty(shape).uniform_(-0.5, 0.5, generator=torch.Generator().manual_seed(6)) if stochastic else None
    ref = O.grad_quantize(g, 8, noise)
    Q.GRAD_NOISE[0] = lambda like: noise.to(like.device)
    try:
        got = Q.quantize_grad_tensor(g.to(gpu), 8, stochastic=stochastic).cpu()
    finally:
        Q.GRAD_NOISE[0] = Q.grad_noise
    assert torch.equal(got, ref)


def test_grad_quantizer_unbiased_draw(gpu):
    """The default draw is torch's uniform(-0.5, 0.5) on the device: stochastic rounding is
    unbiased -- the mean of many quantizations of one gradient approaches the gradient."""
    g = torch.randn(4096, generator=torch.Generator().manual_seed(8)).to(gpu)
    acc = torch.zeros_like(g)
    for _ in range(64):
        acc += Q.quantize_grad_tensor(g, 8)
    step = (float(g.max()) - float(g.min())) / 255.0
    assert (acc / 64 - g).abs().max().item() < 0.5 * step


@pytest.mark.parametrize("name", TRAIN)
def test_layer_train_step_vs_oracle(gpu, name):
    d = load_fixture(name)
    mod = train_params(d).to(gpu).train()
    x = torch.from_numpy(d["x"])
    xg = x.to(gpu).requires_grad_(True)
    gy = torch.from_numpy(d["gy"])
    noise = torch.from_numpy(d["noise"])
    # the batch range the device measures (QuantMeasure train branch, fp64 device reductions)
    mn, mx, _, _ = Q.measure_stats(xg.detach())
    Q.GRAD_NOISE[0] = lambda like: noise.to(like.device)
    try:
        y = mod(xg)
        assert y.requires_grad
        y.backward(gy.to(gpu))
    finally:
        Q.GRAD_NOISE[0] = Q.grad_noise
    xo = x.clone().requires_grad_(True)
    cpu = train_params(d)
    w = cpu.weight.detach().clone().requires_grad_(True)
    b = None if cpu.bias is None else cpu.bias.detach().clone().requires_grad_(True)
    yo = oracle_train(d, xo, w, b, (float(mn), float(mx)))
    yo.backward(gy)

    def close(a, ref, what, rel):
        err = (a.detach().cpu() - ref).abs().max().item()
        assert err <= rel * ref.abs().max().item() + 1e-6, f"{name} {what}: {err}"

    close(y, yo.detach(), "y", 1e-5)
    close(xg.grad, xo.grad, "grad_x", 1e-4)
    close(mod.weight.grad, w.grad, "grad_w", 1e-4)
    if b is not None:
        close(mod.bias.grad, b.grad, "grad_b", 1e-4)
    # the running statistics moved exactly once (train branch side effect, quantize.py:225-236)
    assert float(mod.quantize_input.num_measurements) == 1.0


@pytest.mark.parametrize("name", ["model_resnet18_cifar", "model_mobilenet"])
def test_model_training_step(gpu, name):
    """main.py's train step on a whole quantized model (RangeBN's differentiable statistics,
    straight-through quantizers, 8-bit gradients): every parameter receives a finite, non-zero
    gradient, and one SGD step changes the loss."""
    import torch.nn.functional as F
    from fixtures_util import build_model
    from qnn import synthetic
    d = load_fixture(name)
    model, x = build_model(d)
    model = model.to(gpu).train()
    # batch 16: RangeBN's training statistics split B*H*W into 16 chunks (quantize.py:468), also
    # on MobileNet's 7x7 maps and the 1-D RangeBN after a linear layer
    xg = synthetic.input_batch((16,) + tuple(x.shape[1:]), 21).to(gpu)
    tgt = torch.arange(16, device=gpu) % 10
    loss = F.cross_entropy(model(xg), tgt)
    loss.backward()
    for n, p in model.named_parameters():
        assert p.grad is not None, n
        assert torch.isfinite(p.grad).all(), n
        assert p.grad.abs().sum().item() > 0, n
    with torch.no_grad():
        for p in model.parameters():
            p -= 1e-3 * p.grad
    loss2 = F.cross_entropy(model(xg), tgt)
    assert torch.isfinite(loss2) and loss2.item() != loss.item()
