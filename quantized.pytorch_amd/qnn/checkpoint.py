"""Checkpoints of the reference's training / calibration driver.

The reference saves `{'epoch', 'model', 'config', 'state_dict', 'best_prec1', 'regime'}`
(main.py:196-203, :308-315, utils' save_checkpoint) and, for a quantized model whose
checkpoint lacks the calibrated buffers, `load_maybe_calibrate` (main.py:154-205):
  1. strict `load_state_dict` of the loaded object;
  2. on failure, the `<model>-<depth>.measure` checkpoint next to the run, if present
     (unwrapping 'state_dict', logging 'best_prec1'), loaded strictly;
  3. else a non-strict load, measure mode (set_measure_mode), one pass over calibration
     data, measure mode off, and the `.measure` checkpoint is written.
Here every file is read with `torch.load(weights_only=True)` (tensors, dicts, lists,
strings and numbers only: nothing in a checkpoint executes), the calibration pass runs
the device statistics kernels (qnn_measure_stats_f32 / qnn_rangebn_stats_f32) and is
merged across ranks with one all-reduce when a process group is up, and the int8
operands of every QConv2d / QLinear are packed once at load time (`prepack`) instead of
inside the first forward.
"""
import logging
import os

import torch

from .quantize import QConv2d, QLinear, set_measure_mode, use_s2d

__all__ = ["load_checkpoint", "save_checkpoint", "measure_name", "prepack", "load_maybe_calibrate"]

log = logging.getLogger("qnn.checkpoint")


def load_checkpoint(path):
    """(state_dict, meta) of a reference checkpoint file: a bare state_dict or the
    {'state_dict', ...} wrapper (main.py:165-167).  Weights-only: refuses anything
    that would need unpickling code."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and "state_dict" in obj:
        meta = {k: v for k, v in obj.items() if k != "state_dict"}
        return obj["state_dict"], meta
    if not isinstance(obj, dict):
        raise ValueError(f"qnn: {path} holds a {type(obj).__name__}, not a state_dict or checkpoint dict")
    return obj, {}


def save_checkpoint(path, model, model_name="", config="", best_prec1=0.0, epoch=0, regime=None):
    """The reference's checkpoint dict (main.py:196-203) with tensors on the CPU."""
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save({"epoch": epoch, "model": model_name, "config": config, "state_dict": sd,
                "best_prec1": float(best_prec1), "regime": regime}, path)


def measure_name(model_name, depth):
    """'<model>-<depth>.measure' (main.py:158)."""
    return f"{model_name}-{depth}.measure"


def prepack(model):
    """Pack the int8 operands of every QConv2d / QLinear on its device now (the variant
    its forward uses: depthwise, space-to-depth stem or implicit GEMM), so the first
    forward does no packing.  Returns the number of layers packed."""
    n = 0
    for m in model.modules():
        if isinstance(m, QConv2d):
            if m.groups > 1 and m.groups == m.in_channels == m.out_channels:
                m._pack(depthwise=True)
            else:
                m._pack(s2d=use_s2d(m.in_channels // m.groups, m.kernel_size[0], m.stride))
            n += 1
        elif isinstance(m, QLinear):
            m._pack()
            n += 1
    return n


def _to_device(model, device):
    return model.to(device) if device is not None else model


def load_maybe_calibrate(model, checkpoint, save_dir, model_name, depth, calib_batches=None, device=None,
                         pack=True):
    """main.py:154-205 for a quantized model.  `checkpoint`: a path or a state_dict.
    Returns one of 'checkpoint' (strict load), 'measure' (the saved .measure), or
    'calibrated' (measure-mode pass over `calib_batches`, then the .measure written).
    The model ends on `device`, in eval mode, pre-packed unless pack=False."""
    sd = load_checkpoint(checkpoint)[0] if isinstance(checkpoint, (str, os.PathLike)) else checkpoint
    how = "checkpoint"
    try:
        model.load_state_dict(sd)
    except (RuntimeError, KeyError) as e:
        mpath = os.path.join(save_dir, measure_name(model_name, depth))
        if os.path.exists(mpath):
            msd, meta = load_checkpoint(mpath)
            if "best_prec1" in meta:
                log.info("measured checkpoint loaded, reference score top1 %.3f", meta["best_prec1"])
            model.load_state_dict(msd)
            how = "measure"
        else:
            if calib_batches is None:
                raise RuntimeError(f"qnn: checkpoint lacks calibrated buffers and no {mpath} exists; "
                                   "pass calib_batches to calibrate") from e
            model.load_state_dict(sd, strict=False)
            model = _to_device(model, device)
            # the reference calibrates a freshly built (train-mode) model; set_measure_mode
            # then puts BatchNorm layers into eval (main.py:182, quantize.py:547-552)
            model.train()
            set_measure_mode(model, True)
            with torch.no_grad():
                for x in calib_batches:
                    model(x.to(next(model.parameters()).device))
            set_measure_mode(model, False)
            from . import dist as qdist
            # weighted by this rank's samples per calibration batch (ragged shards merge exactly)
            nb = len(calib_batches)
            qdist.allreduce_calibration(model, samples=sum(int(x.shape[0]) for x in calib_batches) / nb if nb else 0)
            if not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0:
                save_checkpoint(mpath, model, model_name=model_name, config=str({"depth": depth}))
            how = "calibrated"
    model = _to_device(model, device)
    model.eval()
    if pack:
        prepack(model)
    return how
