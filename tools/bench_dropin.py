#!/usr/bin/env python3
"""The drop-in module boundary, measured: quantize + convolve (two launches) against the fused
quantize-on-load convolution (qnn_qconv2d_fwd_nchw_f32, one launch).

The reference's QConv2d.forward (/root/reference/models/modules/quantize.py:314-354) takes an fp32
NCHW input and quantizes it before the conv; here that is qnn_quantize_nchw_to_nhwc8 then
qnn_qconv2d_fwd, or one persistent-band launch that quantizes each input band into LDS.

Per layer (one JSON line each): HIP-event medians of every launch of both paths, over `--reps`
forwards of the module (the two-launch conv at its autotuned tile, the fused launch at every
persistent-band configuration that fits: the fastest and the default), the whole module forward
wall time both ways, and the algorithmic bytes.  Then the module path of whole models (ResNet-18
b128, ResNet-50 b256) in images/s with the fused input off and on, timed as bench.py times
`module_path_images_per_s`.  Outputs are checked bitwise equal between the paths on every layer.

  python tools/bench_dropin.py --out gpurun_out/r5_bench_layers_dropin.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quantized.pytorch_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from qnn import _lib, synthetic  # noqa: E402
from qnn import quantize as Q  # noqa: E402

# (name, cin, cout, stride, batch, hw)
LAYERS = [
    ("r18_layer1_3x3_64_56_b128", 64, 64, 1, 128, 56),
    ("r18_layer2_entry_3x3s2_64_128_56_b128", 64, 128, 2, 128, 56),
    ("r18_layer2_3x3_128_28_b128", 128, 128, 1, 128, 28),
    ("r50_layer1_3x3_64_56_b256", 64, 64, 1, 256, 56),
    ("headline_r50_layer3_3x3_256_14_b256", 256, 256, 1, 256, 14),
    ("r18_layer4_3x3_512_7_b128", 512, 512, 1, 128, 7),
]
NAMES = ("qnn_quantize_nchw_to_nhwc8", "qnn_qconv2d_fwd", "qnn_qconv2d_fwd_nchw_f32")


def _timed(wrap, x, reps):
    """(median ms per launch name, median module wall ms, output)."""
    t = _lib.LaunchTimer(NAMES)
    walls = []
    with torch.no_grad():
        y = wrap(x)  # warm (autotune, packing, tables)
        torch.cuda.synchronize()
        _lib.set_timer(t)
        try:
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                y = wrap(x)
                e1.record()
                walls.append((e0, e1))
        finally:
            _lib.set_timer(None)
        torch.cuda.synchronize()
    per = {}
    for n, ms in t.durations_ms():
        per.setdefault(n, []).append(ms)
    return ({n: float(np.median(v)) for n, v in per.items()},
            float(np.median([a.elapsed_time(b) for a, b in walls])), y.clone())


def layer_row(name, cin, cout, st, n, hw, reps, dev):
    m = Q.QConv2d(cin, cout, 3, stride=st, padding=1, bias=False, num_bits_grad=8, biprecision=True)
    wrap = nn.Sequential(m)
    synthetic.init_params(wrap, 5)
    m.quantize_input.running_min.fill_(0.0)
    m.quantize_input.running_max.fill_(2.75)
    wrap = wrap.to(dev).eval()
    x = (synthetic.input_batch((n, cin, hw, hw), 9, relu=True) * 1.1).to(dev)
    ho = (hw + 2 - 3) // st + 1
    row = {"layer": name, "cin": cin, "cout": cout, "stride": st, "batch": n, "hw": hw,
           "algorithmic_bytes": {"input_f32": 4 * n * cin * hw * hw, "codes_i8": n * (hw + 2) ** 2 * m._pack().cin_pad,
                                 "weights_i8": cout * 9 * cin, "output_f32": 4 * n * cout * ho * ho}}
    # two launches, the conv at its autotuned tile (the strongest two-launch baseline)
    Q.MODULE_AUTOTUNE[0] = True
    m.qnn_fused_input = False
    per2, wall2, y2 = _timed(wrap, x, reps)
    Q.MODULE_AUTOTUNE[0] = False
    row["two_launch"] = {"quantize_ms": per2.get(NAMES[0]), "conv_ms": per2.get(NAMES[1]),
                         "sum_ms": (per2.get(NAMES[0]) or 0) + (per2.get(NAMES[1]) or 0), "module_wall_ms": wall2,
                         "conv_tile": int(m._last_conv[0].tile) - 1}
    fused = {}
    for k in _lib.tile_ids("qconv_pb_kernel"):
        m.qnn_fused_input, m.qnn_fused_tile = True, k + 1
        perf, wallf, yf = _timed(wrap, x, reps)
        if not m._last_fused:
            continue
        fused[k] = {"fused_ms": perf.get(NAMES[2]), "module_wall_ms": wallf, "bitwise_equal": bool(torch.equal(yf, y2))}
    m.qnn_fused_input, m.qnn_fused_tile = True, 0
    perd, walld, yd = _timed(wrap, x, reps)
    m.qnn_fused_input, m.qnn_fused_tile = None, 0
    if fused:
        best = min(fused, key=lambda k: fused[k]["fused_ms"])
        row["fused"] = {"per_config": {str(k): v for k, v in fused.items()}, "best_config": best,
                        "best_ms": fused[best]["fused_ms"], "default_ms": perd.get(NAMES[2]),
                        "default_module_wall_ms": walld, "bitwise_equal": bool(torch.equal(yd, y2)) and
                        all(v["bitwise_equal"] for v in fused.values())}
        row["speedup_launch_sum"] = row["two_launch"]["sum_ms"] / fused[best]["fused_ms"]
        fb = row["algorithmic_bytes"]
        row["fused_hbm_gbs"] = (fb["input_f32"] + fb["weights_i8"] + fb["output_f32"]) / (fused[best]["fused_ms"] * 1e6)
    else:
        row["fused"] = None
        row["fused_note"] = ("no persistent-band configuration fits (3x3 on 64 or 128 padded input channels only): "
                             "the module takes the two-launch path; the quantize launch bounds any fusion's gain")
        row["fusion_gain_bound"] = row["two_launch"]["sum_ms"] / row["two_launch"]["conv_ms"]
    return row


def model_row(depth, batch, steps, dev):
    import bench
    model = bench.build(dev, depth)
    x = synthetic.input_batch((batch, 3, 224, 224), 21).to(dev)
    out = {"model": f"resnet{depth}", "batch": batch}
    ys = {}
    for fused in (False, True):
        Q.FUSED_INPUT[0] = fused
        with torch.no_grad():
            for _ in range(2):
                model(x)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(steps):
                y = model(x)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t1
        ys[fused] = y.clone()
        n_fused = sum(1 for mm in model.modules() if isinstance(mm, Q.QConv2d) and mm._last_fused)
        out["fused" if fused else "two_launch"] = {"module_path_images_per_s": batch * steps / dt,
                                                   "convs_fused": n_fused}
    Q.FUSED_INPUT[0] = False
    out["bitwise_equal"] = bool(torch.equal(ys[False], ys[True]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/r5_bench_layers_dropin.jsonl")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--no-models", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        for spec in LAYERS:
            row = layer_row(*spec, a.reps, dev)
            print(json.dumps(row), flush=True)
            f.write(json.dumps(row) + "\n")
            f.flush()
        if not a.no_models:
            for depth, batch in ((18, 128), (50, 256)):
                row = model_row(depth, batch, a.steps, dev)
                print(json.dumps(row), flush=True)
                f.write(json.dumps(row) + "\n")
                f.flush()


if __name__ == "__main__":
    main()
