#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the survey/build container, where /root/reference exists.  It imports
the reference's hot-path files through `tools/refload.py` (in-memory stubs for
the un-vendored `utils` submodule and torchvision), builds reference modules,
fills their parameters from this package's deterministic numpy initializer
(`qnn/synthetic.py`), calibrates them exactly as `main.py:154-205` does
(`set_measure_mode(True)`, train-mode forwards, `set_measure_mode(False)`), and
records the reference's eval outputs.

Fixtures hold data only (numpy .npz, loadable with allow_pickle=False):
  * quantize_kat.npz   - UniformQuantize known answers (float-range, tensor-range,
                         None-range paths; ties, clamps, min==max, negative ranges)
  * layer_<name>.npz   - one QConv2d / QLinear / RangeBN each: calibrated buffers,
                         eval output; weights and inputs are rebuilt from seeds
                         (checksums stored to catch drift)
  * model_<name>.npz   - whole-model logits (cifar/imagenet ResNet-18, ResNet-50,
                         MobileNet) + every calibrated buffer

The files are byte-for-byte reproducible (`savez`: fixed zip metadata; every input from
seeds): tools/check_golden.sh regenerates into a scratch directory and compares hashes.

Note on weight_min/weight_max (and bias_min/bias_max): in measure mode the reference skips
the block that refreshes them (enable_quant is False, quantize.py:316-330), so after
calibration they still hold the min/max of torch's default initialisation under
torch.manual_seed(0) -- which is what the fixtures record; eval forwards recompute them.

Usage: python tools/gen_golden.py [--only NAME ...] [--out DIR]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "quantized.pytorch_amd"))

import refload  # noqa: E402
from qnn import synthetic  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")


def savez(path, **arrays):
    """np.savez_compressed with reproducible bytes: fixed zip timestamps and modes, entries
    in insertion order (numpy's own writer stamps the current time).  np.load reads it."""
    import io
    import zipfile
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as zf:
        for k, v in arrays.items():
            buf = io.BytesIO()
            np.lib.format.write_array(buf, np.asanyarray(v), allow_pickle=False)
            zi = zipfile.ZipInfo(k + ".npy", date_time=(1980, 1, 1, 0, 0, 0))
            zi.compress_type = zipfile.ZIP_DEFLATED
            zi.external_attr = 0o644 << 16
            zf.writestr(zi, buf.getvalue())

# --------------------------------------------------------------------------- layers
# (name, kind, ctor kwargs, input shape, calib relu?, eval relu?)
LAYERS = [
    ("c3x3_64_64_s1", "conv", dict(in_channels=64, out_channels=64, kernel_size=3, stride=1, padding=1, bias=False), (2, 64, 8, 8), True),
    ("c3x3_64_128_s2", "conv", dict(in_channels=64, out_channels=128, kernel_size=3, stride=2, padding=1, bias=False), (2, 64, 16, 16), True),
    ("c1x1_256_64", "conv", dict(in_channels=256, out_channels=64, kernel_size=1, bias=False), (2, 256, 8, 8), True),
    ("c1x1_64_128_s2", "conv", dict(in_channels=64, out_channels=128, kernel_size=1, stride=2, bias=False), (2, 64, 8, 8), True),
    ("c7x7_3_64_s2", "conv", dict(in_channels=3, out_channels=64, kernel_size=7, stride=2, padding=3, bias=False), (2, 3, 32, 32), False),
    ("c3x3_3_32_s2", "conv", dict(in_channels=3, out_channels=32, kernel_size=3, stride=2, padding=1, bias=False), (2, 3, 32, 32), False),
    ("dw3x3_32_s1_bias", "conv", dict(in_channels=32, out_channels=32, kernel_size=3, stride=1, padding=1, groups=32, bias=True), (2, 32, 16, 16), True),
    ("dw3x3_64_s2_bias", "conv", dict(in_channels=64, out_channels=64, kernel_size=3, stride=2, padding=1, groups=64, bias=True), (2, 64, 16, 16), True),
    ("c3x3_16_16_cifar", "conv", dict(in_channels=16, out_channels=16, kernel_size=3, stride=1, padding=1, bias=False), (2, 16, 32, 32), True),
    ("c3x3_512_512_k4608", "conv", dict(in_channels=512, out_channels=512, kernel_size=3, stride=1, padding=1, bias=False), (2, 512, 7, 7), True),
    ("c3x3_24_40_ragged", "conv", dict(in_channels=24, out_channels=40, kernel_size=3, stride=1, padding=1, bias=False), (3, 24, 9, 11), True),
    ("c3x3_64_64_aciq", "conv_aciq", dict(in_channels=64, out_channels=64, kernel_size=3, stride=1, padding=1, bias=False), (2, 64, 8, 8), True),
    ("fc_512_1000", "linear", dict(in_features=512, out_features=1000, bias=True), (4, 512), True),
    ("fc_64_10", "linear", dict(in_features=64, out_features=10, bias=True), (4, 64), True),
    ("rbn_32", "rangebn", dict(num_features=32), (4, 32, 8, 8), False),
]
BIPREC = dict(num_bits=8, num_bits_weight=8, num_bits_grad=8, biprecision=True)

# (name, factory, kwargs, eval batch shape, calib batch)
MODELS = [
    ("resnet18_cifar", "resnet", dict(depth=18, dataset="cifar10"), (8, 3, 32, 32), 16),
    ("resnet18_imagenet", "resnet", dict(depth=18, dataset="imagenet"), (2, 3, 224, 224), 16),
    ("resnet50_imagenet", "resnet", dict(depth=50, dataset="imagenet"), (2, 3, 224, 224), 16),
    ("mobilenet", "mobilenet", dict(), (2, 3, 224, 224), 16),
]


def calibrate(Q, model, batches):
    Q.set_measure_mode(model, True)
    model.train()
    with torch.no_grad():
        for b in batches:
            model(b)
    Q.set_measure_mode(model, False)
    model.eval()


def buffers(model):
    return {"buf/" + k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()
            if not any(k.endswith(s) for s in (".weight", ".bias")) or "running" in k}


def gen_quantize_kat(Q):
    rec = {}
    # float-range path (QuantMeasure eval: float(min), float(max)), quantize.py:249
    ranges = [(-2.5, 3.1), (0.0, 6.0), (-1e-3, 1e-3), (1.0, 1.0), (-5.0, -1.0), (0.0, 0.0), (-0.3, 12.7)]
    for i, (mn, mx) in enumerate(ranges):
        mn, mx = float(np.float32(mn)), float(np.float32(mx))
        rng = synthetic._gen(1000, i)
        x = (rng.standard_normal(4096) * max(abs(mn), abs(mx), 1.0) * 1.3 + (mn + mx) / 2).astype(np.float32)
        s = max((mx - mn) / 255.0, 1e-8)
        ks = np.arange(0, 256, dtype=np.float64)
        ties = np.concatenate([mn + (ks + 0.5 + d) * s for d in (-1e-6, 0.0, 1e-6)]).astype(np.float32)
        edge = np.array([mn, mx, mn - 1e3, mx + 1e3, 0.0, -0.0, mn + s * 255.5, mn - s * 0.5], dtype=np.float32)
        x = np.concatenate([x, ties, edge]).astype(np.float32)
        y = Q.quantize(torch.from_numpy(x), 8, mn, mx).numpy()
        rec[f"float/{i}/x"] = x
        rec[f"float/{i}/range"] = np.array([mn, mx], dtype=np.float64)
        rec[f"float/{i}/y"] = y
    # tensor-range per-output-channel path (QConv2d weights), quantize.py:317-334
    for i, shape in enumerate([(64, 64, 3, 3), (40, 24, 3, 3), (32, 1, 3, 3), (10, 64)]):
        w = synthetic.normal(shape, 2000, i, 0.05)
        w[0] = 0.0  # a constant channel: scale floor 1e-8
        wt = torch.from_numpy(w)
        sh = (shape[0],) + (1,) * (len(shape) - 1)
        wmin = wt.flatten(1).min(-1)[0].view(sh)
        wmax = wt.flatten(1).max(-1)[0].view(sh)
        y = Q.quantize(wt, 8, wmin, wmax).numpy()
        rec[f"tensor/{i}/x"] = w
        rec[f"tensor/{i}/y"] = y
    # None-range path (RangeBN bias), quantize.py:45-55, :498
    for i, n in enumerate([32, 64, 1000]):
        b = synthetic.uniform((n,), -0.1, 0.3, 3000, i)
        rec[f"none/{i}/x"] = b
        rec[f"none/{i}/y"] = Q.quantize(torch.from_numpy(b), num_bits=8).numpy()
    savez(os.path.join(OUT, "quantize_kat.npz"), **rec)
    print("quantize_kat:", len(rec), "arrays")


def gen_layer(Q, name, kind, kw, shape, relu_in):
    torch.manual_seed(0)
    if kind in ("conv", "conv_aciq"):
        mod = Q.QConv2d(**kw, **BIPREC)
    elif kind == "linear":
        mod = Q.QLinear(**kw, **BIPREC)
    else:
        mod = Q.RangeBN(kw["num_features"], num_bits=8, num_bits_grad=8)
    wrap = nn.Sequential(mod)
    synthetic.init_params(wrap, seed=7)
    cal = [synthetic.input_batch(shape, 100 + j, relu=relu_in) for j in range(2)]
    calibrate(Q, wrap, cal)
    if kind == "conv_aciq":
        Q.set_global_quantization_method(wrap, "aciq")
    x = synthetic.input_batch(shape, 200, relu=relu_in) * 1.25  # exceed the calibrated range a bit
    bufs = buffers(wrap)  # before the eval forward (aciq mutates running_var in place, quantize.py:258)
    with torch.no_grad():
        y = wrap(x)
    rec = {"config": np.array(json.dumps(dict(kind=kind, kw=kw, shape=shape, relu_in=relu_in,
                                                param_seed=7, calib_seeds=[100, 101], eval_seed=200,
                                                eval_scale=1.25))),
           "y": y.numpy(), "param_checksum": np.array(synthetic.param_checksum(wrap)),
           "x_checksum": np.array(float(x.double().abs().sum()))}
    rec.update(bufs)
    savez(os.path.join(OUT, f"layer_{name}.npz"), **rec)
    print(f"layer_{name}: y{tuple(y.shape)} max|y|={y.abs().max():.4g}")


def gen_model(Q, RQ, MQ, name, fac, kw, shape, calib_b):
    torch.manual_seed(0)
    model = RQ.resnet_quantized(**kw) if fac == "resnet" else MQ.mobilenet_quantized(**kw)
    synthetic.init_params(model, seed=11)
    cal_shape = (calib_b,) + tuple(shape[1:])
    cal = [synthetic.input_batch(cal_shape, 300 + j) for j in range(2)]
    calibrate(Q, model, cal)
    x = synthetic.input_batch(shape, 400)
    bufs = buffers(model)
    with torch.no_grad():
        logits = model(x)
    rec = {"config": np.array(json.dumps(dict(factory=fac, kw=kw, shape=shape, param_seed=11,
                                                calib_seeds=[300, 301], calib_batch=calib_b,
                                                eval_seed=400))),
           "logits": logits.numpy(), "param_checksum": np.array(synthetic.param_checksum(model)),
           "keys": np.array(list(model.state_dict().keys()))}
    rec.update(bufs)
    savez(os.path.join(OUT, f"model_{name}.npz"), **rec)
    print(f"model_{name}: logits{tuple(logits.shape)} argmax={logits.argmax(1).tolist()}")


# training-side fixtures: (name, kind, kwargs, input shape, num_bits_grad, biprecision)
TRAIN = [
    ("train_c3x3_biprec", "conv", dict(in_channels=16, out_channels=32, kernel_size=3, stride=1, padding=1, bias=True),
     (2, 16, 8, 8), 8, True),
    ("train_c3x3_gradq", "conv", dict(in_channels=16, out_channels=32, kernel_size=3, stride=2, padding=1, bias=True),
     (2, 16, 9, 9), 8, False),
    ("train_c3x3_plain", "conv", dict(in_channels=16, out_channels=16, kernel_size=3, stride=1, padding=1, bias=False),
     (2, 16, 8, 8), None, False),
    ("train_fc_biprec", "linear", dict(in_features=64, out_features=10, bias=True), (4, 64), 8, True),
]


def gen_train(Q, name, kind, kw, shape, nbg, biprec):
    """One reference QConv2d / QLinear in training mode: forward on a fresh batch (QuantMeasure
    batch statistics), backward of a fixed output gradient.  The stochastic rounding draw of the
    gradient quantizer is torch's first CPU draw after manual_seed(NOISE_SEED); it is stored too,
    so a device run can be fed the same noise."""
    torch.manual_seed(0)
    args = dict(num_bits=8, num_bits_weight=8, num_bits_grad=nbg, biprecision=biprec)
    mod = Q.QConv2d(**kw, **args) if kind == "conv" else Q.QLinear(**kw, **args)
    wrap = nn.Sequential(mod)
    synthetic.init_params(wrap, seed=9)
    wrap.train()
    x = synthetic.input_batch(shape, 500).requires_grad_(True)
    y = wrap(x)
    gy = synthetic.input_batch(tuple(y.shape), 501)
    NOISE_SEED = 1234
    torch.manual_seed(NOISE_SEED)
    noise = torch.empty(tuple(y.shape)).uniform_(-0.5, 0.5)
    torch.manual_seed(NOISE_SEED)  # the reference's backward draws exactly this
    y.backward(gy)
    rec = {"config": np.array(json.dumps(dict(kind=kind, kw=kw, shape=shape, num_bits_grad=nbg, biprecision=biprec,
                                                param_seed=9, x_seed=500, gy_seed=501, noise_seed=NOISE_SEED))),
           "x": x.detach().numpy(), "y": y.detach().numpy(), "gy": gy.numpy(), "noise": noise.numpy(),
           "grad_x": x.grad.numpy(), "grad_w": mod.weight.grad.numpy(),
           "param_checksum": np.array(synthetic.param_checksum(wrap))}
    if mod.bias is not None:
        rec["grad_b"] = mod.bias.grad.numpy()
    rec.update(buffers(wrap))
    savez(os.path.join(OUT, f"{name}.npz"), **rec)
    print(f"{name}: y{tuple(y.shape)} |grad_x|={x.grad.abs().sum():.6g} |grad_w|={mod.weight.grad.abs().sum():.6g}")


def main():
    global OUT
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--out", default=OUT, help="output directory (default tests/golden)")
    a = ap.parse_args()
    OUT = a.out
    torch.set_num_threads(max(1, min(8, os.cpu_count() or 1)))
    Q, RQ, MQ = refload.load()
    os.makedirs(OUT, exist_ok=True)
    want = set(a.only or [])
    if not want or "quantize_kat" in want:
        gen_quantize_kat(Q)
    for L in LAYERS:
        if not want or L[0] in want:
            gen_layer(Q, *L)
    for M in MODELS:
        if not want or M[0] in want:
            gen_model(Q, RQ, MQ, *M)
    for T in TRAIN:
        if not want or T[0] in want:
            gen_train(Q, *T)


if __name__ == "__main__":
    main()
