#!/usr/bin/env python3
"""Benchmark: images/sec of the 8-bit ResNet-18 eval forward on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]): resnet_quantized depth=18, ImageNet shape
3x224x224, batch 128 per GPU, int8 MFMA path, synthetic inputs resident in HBM.
A "step" is one forward of one batch (plus, at N>1, the RCCL gather of the
logits to rank 0, issued asynchronously and drained inside the timed region).  Weak scaling: every rank processes its own 128 images.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line (see DESIGN.md §Measurement for every field).
"""
import argparse
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "quantized.pytorch_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec, 8-bit ResNet-18 224×224 @1/2/4/8 GPU; % int8-MFMA roofline"
ROUND = 6  # profiles/rNN_traffic_* from an earlier round measured other kernels: never cited as traffic
PEAK_INT8_TOPS = 5000.0   # dense int8 MFMA, 256 CU x 2.4 GHz (MI355X_MICROARCH.md: 2x bf16 2.5 PF)
PEAK_HBM_GBS = 8000.0


def model_ops(model, batch, hw=224):
    """Algorithmic int8 ops per forward: sum over QConv2d/QLinear of 2*N*Cout*Ho*Wo*Cin/g*kh*kw
    (SURVEY.md §8(d)); returned as (total, mfma_part) where mfma_part excludes depthwise."""
    from qnn.quantize import QConv2d, QLinear
    shapes = {}
    hooks = []

    def rec(m, inp, out):
        shapes[m] = (tuple(inp[0].shape), tuple(out.shape))

    for m in model.modules():
        if isinstance(m, (QConv2d, QLinear)):
            hooks.append(m.register_forward_hook(rec))
    with torch.no_grad():
        model(torch.zeros(1, 3, hw, hw, device=next(model.parameters()).device))
    for h in hooks:
        h.remove()
    total = mfma = 0
    for m, (ishape, oshape) in shapes.items():
        if isinstance(m, QLinear):
            ops = 2 * batch * m.out_features * m.in_features
        else:
            kh, kw = m.kernel_size
            ops = 2 * batch * m.out_channels * oshape[2] * oshape[3] * (m.in_channels // m.groups) * kh * kw
        total += ops
        if isinstance(m, QLinear) or m.groups == 1:
            mfma += ops
    return total, mfma


def calibrate(model, device, seed, batches=2, bsz=16):
    from qnn import synthetic
    from qnn.quantize import set_measure_mode
    set_measure_mode(model, True)
    model.train()
    with torch.no_grad():
        for j in range(batches):
            model(synthetic.input_batch((bsz, 3, 224, 224), seed + j).to(device))
    set_measure_mode(model, False)
    model.eval()


def build(device, depth, seed=11, arch="resnet"):
    from qnn import synthetic
    torch.manual_seed(0)
    if arch == "mobilenet":
        from qnn.mobilenet_quantized import mobilenet_quantized
        model = mobilenet_quantized()
    else:
        from qnn.resnet_quantized import resnet_quantized
        model = resnet_quantized(depth=depth, dataset="imagenet")
    synthetic.init_params(model, seed)
    model = model.to(device)
    calibrate(model, device, 300)
    return model


def cpu_model_name():
    """The host CPU model (lscpu's "Model name", from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_threads():
    """(threads used, affinity cores): every core of this process's affinity mask, capped
    at the box's CPU share (OMP_NUM_THREADS, set to the per-GPU share on the GPU box,
    where the affinity mask spans the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", aff) or aff)
    return max(1, min(aff, share)), aff


def cpu_baseline(model_cpu_sd, depth, batch, iters, threads, arch="resnet", warmup=2, config_batch=None):
    """Oracle (the reference's fake-quant CPU forward, restated and pinned bitwise to it)
    on a bounded sample: `warmup` untimed forwards, then the median of
    `iters`, with the reference's biprecision double contraction and, separately, one
    contraction per layer."""
    from oracle import qnn_oracle as O
    from qnn import synthetic
    torch.set_num_threads(threads)
    x = synthetic.input_batch((batch, 3, 224, 224), 4242)
    sd = {k: v.clone() for k, v in model_cpu_sd.items()}
    kw = dict(depth=depth, dataset="imagenet") if arch == "resnet" else {}

    def median_s(biprecision):
        with O.contraction(biprecision=biprecision):
            for _ in range(warmup):
                O.model_forward(sd, x, arch, kw)
            times = []
            for _ in range(iters):
                t0 = time.perf_counter()
                O.model_forward(sd, x, arch, kw)
                times.append(time.perf_counter() - t0)
        return float(np.median(times))

    med, med1 = median_s(True), median_s(False)
    cb = config_batch or batch
    return {"value": round(batch / med, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle/qnn_oracle.py {model_name(arch, depth)} imagenet fake-quant forward (biprecision "
                      f"double conv, as the reference), batch {batch}, median of {iters} after {warmup} warm-ups, "
                      f"torch {torch.__version__} CPU, {threads} threads",
            "cpu_model": cpu_model_name(), "affinity_cores": len(os.sched_getaffinity(0)),
            "batch": batch, "s_per_batch": round(med, 4),
            "extrapolation": None if cb == batch else
            f"images/s measured at batch {batch}, reported for the batch-{cb} config: the CPU forward is a "
            f"sequence of batched ops whose time is linear in the batch (per-image rate)",
            "single_conv": {"value": round(batch / med1, 3), "unit": "images/s", "s_per_batch": round(med1, 4),
                            "note": "one contraction per layer instead of the reference's out1 + out2 - out1"}}


def timed_run(step, steps, warmup, world, sync=None):
    """The contract's timed region: `warmup` untimed steps, then barrier + sync, exactly
    `steps` steps, every step's in-flight gather drained (`.result()`), barrier + sync;
    returns the MAX over ranks of the elapsed seconds.  `step()` returns a
    ShardedInference handle (or None); `sync` is the device synchronize (None on CPU)."""
    sync = sync or (lambda: None)

    def fence():
        sync()
        if world > 1:
            dist.barrier()
        sync()

    with torch.no_grad():
        for h in [step() for _ in range(warmup)]:
            if h is not None:
                h.result()
        fence()
        t0 = time.perf_counter()
        for h in [step() for _ in range(steps)]:
            if h is not None:
                h.result()
        fence()
        elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def throughput(global_batch, steps, elapsed):
    """Whole-job images/s: every rank's images of every timed step over the slowest rank's time."""
    return global_batch * steps / elapsed


# the contractions, and the split residual-chain epilogue of a block's last conv (Engine
# split_chain): epilogue work moved out of a conv launch is still charged to the contractions
CONV_LAUNCHES = ("qnn_qconv2d_fwd", "qnn_qconv2d_maxpool_fwd", "qnn_chain_epilogue")


def _graph_ms(engine, names, reps):
    """ms per replay of the hipGraph of `names`' launches in plan order (HIP events on torch's
    current stream, the stream the replay runs on)."""
    g, _n = engine.capture_subset(names)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    del g
    return e0.elapsed_time(e1) / reps


def in_graph_times(engine, reps):
    """In-graph kernel time per forward of each launch kind, measured live with HIP events:
    the launches of one kind (every contraction, or every depthwise conv, ...) are captured in
    plan order as a hipGraph of their own, which is replayed `reps` times between two events
    recorded on torch's current stream (the stream the replay runs on).  Each launch thus runs
    once per replay, in plan order and on the engine's own buffers -- no back-to-back repeats
    of one launch over warm operands -- but WITHOUT the other launch kinds in between (input
    quantizer, pooling, depthwise ...), so the L2 / Infinity-Cache contents a launch meets are
    not exactly those of the full graph.

    The contractions' time is the full forward's graph (the engine's own hipGraph, with each
    residual block's downsample conv concurrent with the main path) minus the graph of every
    other launch kind (`conv_ms`): where the other kinds are a large share of the forward (MobileNet's
    depthwise convs feed every pointwise conv through L2), the contraction-only graph reads
    those inputs from HBM instead and runs ~9 % slower than the same launches in the full
    graph; the difference keeps them in their place.  It includes the contractions' in-graph
    launch boundaries (~1 us each), so it bounds their rate from below.  tools/trace_check.py
    cross-checks it against the full-graph trace of the same command.  Returns ({kind: ms per
    forward, each alone}, conv ms, contraction-only graph ms)."""
    out = {name: _graph_ms(engine, [name], reps) for name in dict.fromkeys(engine.launch_names)}
    conv_names = [n for n in CONV_LAUNCHES if n in out]
    other = [n for n in out if n not in conv_names]
    conv_alone = _graph_ms(engine, conv_names, reps)
    if not other:
        return out, conv_alone, conv_alone
    if engine.graph is not None:  # the forward itself (its residual-branch forks included)
        engine.graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            engine.graph.replay()
        e1.record()
        e1.synchronize()
        full = e0.elapsed_time(e1) / reps
    else:
        full = _graph_ms(engine, list(out), reps)
    rest = _graph_ms(engine, other, reps)
    return out, full - rest, conv_alone


def baseline_config(arch, depth, batch, world):
    """Which BASELINE.json config this run measures (C1 is the reference's CPU case)."""
    if arch == "mobilenet":
        return "C4" if batch == 512 and world == 1 else None
    if depth == 18 and batch == 128 and world == 1:
        return "C2"
    if depth == 50 and batch == 256:
        return "C3" if world == 1 else "C5" if world == 8 else f"C5 shape at {world} GPUs"
    return None


def model_name(arch, depth):
    return "mobilenet" if arch == "mobilenet" else f"resnet{depth}"


def pmc_traffic(arch, depth, batch):
    """HBM bytes per forward of the conv launches, from the committed rocprofv3 PMC passes of
    this workload (tools/layer_table.py pmc: FETCH_SIZE x2 per the gfx950 correction +
    WRITE_SIZE).  None when no summary for this exact workload is committed; a summary from an
    earlier round than ROUND measured earlier kernels and is reported as stale, never as traffic."""
    import glob
    import re
    paths = glob.glob(os.path.join(HERE, "profiles", f"r*_traffic_{model_name(arch, depth)}_b{batch}.json"))
    if not paths:
        return None
    rnd = lambda p: int(re.search(r"r(\d+)_traffic", os.path.basename(p)).group(1))  # noqa: E731
    latest = max(paths, key=rnd)
    if rnd(latest) < ROUND:
        return {"stale": f"profiles/{os.path.basename(latest)} (round {rnd(latest)} kernels; not this round's)"}
    with open(latest) as f:
        d = json.load(f)
    d["source"] = f"profiles/{os.path.basename(latest)}: " + d["source"]
    return d


def conv_kernels(engine):
    """'qconv_rb_kernel x9, qconv_kernel x8, ...': the device functions of one forward's
    contraction launches (the autotuned tile configurations, qnn_conv_tile_kernel)."""
    import collections
    from qnn import _lib
    c = collections.Counter(_lib.tile_kernel(k) for k, _ in engine.tiles)
    if "qnn_qconv2d_maxpool_fwd" in engine.launch_names:
        c["stem_pool_kernel"] += engine.launch_names.count("qnn_qconv2d_maxpool_fwd")
    return ", ".join(f"{k} x{v}" for k, v in c.most_common())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--model", choices=("resnet", "mobilenet"), default="resnet")
    ap.add_argument("--cpu-batch", type=int, default=32, help="CPU baseline batch (BASELINE.md §4: b32)")
    ap.add_argument("--cpu-iters", type=int, default=5, help="CPU baseline timed forwards (median)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--module-path", type=int, default=1, help="also time the per-module drop-in path (N=1)")
    args = ap.parse_args()

    from qnn import _lib
    from qnn import dist as qdist
    rank, local_rank, world = qdist.init()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    _lib.load()

    model = build(device, args.depth, arch=args.model)
    total_ops, mfma_ops = model_ops(model, args.batch)
    from qnn import synthetic
    engine = qdist.build_engine(model, args.batch)  # rank 0's autotuned tiles on every rank
    engine.input.copy_(synthetic.input_batch((args.batch, 3, 224, 224), 1234 + rank).to(device))
    runner = qdist.ShardedInference(engine, args.batch * world)

    def step():  # one graph replay + the asynchronous logits gather (overlaps the next replay)
        return runner.submit(engine.input)

    elapsed = timed_run(step, args.steps, args.warmup, world, torch.cuda.synchronize)

    per_kernel, conv_ms_per_fwd, conv_alone_ms = in_graph_times(engine, reps=max(10, args.steps))
    launches = engine.num_launches

    module_ips = per_module_ips = None
    if args.module_path and world == 1:
        from qnn import dispatch

        def time_model(n):  # the reference's caller: output = model(inputs) (main.py:359, no_grad :411)
            with torch.no_grad():
                x = engine.input.clone()
                for _ in range(3):  # the dispatch builds its engine when a shape repeats
                    model(x)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(n):
                    model(x)
                torch.cuda.synchronize()
                return args.batch * n / (time.perf_counter() - t1)

        module_ips = time_model(max(5, args.steps))  # qnn/dispatch.py: the cached fused engine
        old = dispatch.DISPATCH[0]
        dispatch.DISPATCH[0] = "off"  # the per-module kernels (fp32 NCHW at every module boundary)
        per_module_ips = time_model(max(2, args.steps // 4))
        dispatch.DISPATCH[0] = old
        dispatch.reset(model)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        achieved = mfma_ops / (conv_ms_per_fwd * 1e-3) / 1e12
        pmc = pmc_traffic(args.model, args.depth, args.batch)
        nconv = sum(1 for n in engine.launch_names if n == "qnn_qconv2d_fwd")
        nstem = sum(1 for n in engine.launch_names if n == "qnn_qconv2d_maxpool_fwd")
        line = {
            "metric": METRIC,
            "value": round(throughput(args.batch * world, args.steps, elapsed), 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": "synthetic (N(0,1) 3x224x224 on device; numpy-PCG64 weights, reference init law)",
            "config": {"workload": (f"resnet_quantized depth={args.depth}" if args.model == "resnet" else
                                    "mobilenet_quantized") + f" imagenet eval forward, fused int8 engine "
                                   f"(hipGraph), per-GPU batch {args.batch}",
                       "baseline_config": baseline_config(args.model, args.depth, args.batch, world),
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "model_gop_per_batch": round(total_ops / 1e9, 2)},
            "roofline": {"bound": "mfma",
                         "kernel": f"int8 contraction launches of one forward ({nconv} qnn_qconv2d_fwd + "
                                   f"{nstem} fused stem): {conv_kernels(engine)}",
                         "achieved": round(achieved, 2), "peak": PEAK_INT8_TOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_INT8_TOPS, 4),
                         "traffic": None if pmc is None or "stale" in pmc else
                         pmc.get("conv_hbm_bytes_per_forward", pmc["hbm_bytes_per_forward"]),
                         "traffic_source": None if pmc is None else pmc.get("source", "stale: " + pmc.get("stale", "")),
                         "kernel_ms_per_forward": round(conv_ms_per_fwd, 4),
                         "kernel_ms_source": "in-graph: the full forward's hipGraph minus the graph of every "
                                             "other launch kind (bench.in_graph_times)",
                         "kernel_ms_contractions_alone": round(conv_alone_ms, 4),
                         "model_frac": round(total_ops / (ms_per_step * 1e-3) / 1e12 / PEAK_INT8_TOPS, 4)},
            "engine": {"launches_per_forward": launches, "hipgraph": True,
                       "kernel_ms_per_forward": {k: round(v, 4) for k, v in per_kernel.items()},
                       "kernel_ms_source": "in-graph: each launch kind captured as its own hipGraph in plan order, "
                                           "replayed between HIP events (bench.in_graph_times)"},
            "module_path_images_per_s": None if module_ips is None else round(module_ips, 1),
            "module_path_note": "the reference's unchanged caller, output = model(inputs) under no_grad "
                                "(main.py:359/411): ResNet/MobileNet.forward runs a cached fused engine "
                                "(qnn/dispatch.py, policy QNN_ENGINE_DISPATCH), bitwise the per-module path",
            "per_module_images_per_s": None if per_module_ips is None else round(per_module_ips, 1),
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline and world == 1:
            threads, _ = cpu_threads()
            sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
            line["cpu_baseline"] = cpu_baseline(sd, args.depth, args.cpu_batch, args.cpu_iters, threads,
                                                arch=args.model, config_batch=args.batch)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
