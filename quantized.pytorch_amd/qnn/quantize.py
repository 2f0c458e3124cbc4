"""Drop-in mirror of models/modules/quantize.py for MI355X (ROCm / gfx950).

Same public surface as the reference: `quantize`,
`quantize_grad`, `QuantNode`, `QuantMeasure`, `QConv2d`, `QLinear`, `RangeBN`,
the tree helpers (`set_measure_mode`, `set_quant_mode`, `overwrite_params`,
`freeze_quant_params`, `set_global_quantization_method`, ...), identical
constructor arguments, buffers and state_dict keys, so reference checkpoints
`load_state_dict(strict=True)` and models/resnet_quantized.py /
models/mobilenet_quantized.py run unchanged on these classes.

Execution model:
* quantized forward (enable_quant, eval or train) on a ROCm device -> the HIP
  C ABI (`include/qnn.h`): int8 MFMA implicit-GEMM conv / GEMM, fp32 epilogue.
  There is no fallback: a missing library raises `QnnLibraryError`, and a CPU
  tensor raises `RuntimeError` (the reference's CPU fake-quant forward is the
  oracle under oracle/, not part of this package).
* measure mode (enable_quant=False) keeps the reference semantics: float conv /
  linear (`F.conv2d`/`F.linear`, quantize.py:350-352, :429-430) and the
  QuantMeasure / RangeBN statistics updates (:225-239, :466-482) in torch ops.
  This is calibration, off the hot path.
* training: with autograd on, the same int8 forward runs inside
  `_QLayerTrain`, whose backward restates the reference's graph -- straight-through
  quantizers (quantize.py:105-109), UniformQuantizeGrad on the output gradient
  (:112-139, `qnn_grad_quant_f32`) and the biprecision split (:142-156).

Host-scalar caching: the reference reads `float(running_min)` on every call
(2 device->host syncs per layer, quantize.py:249).  Here ranges, packed weights
and epilogue vectors are cached and keyed on the tensors' version counters, so a
steady-state eval forward issues no synchronisation.
"""
import ctypes
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_QMEASURE_ALPHA = {2: 2.83, 3: 3.89, 4: 5.03, 5: 6.2, 6: 7.41, 7: 8.64, 8: 9.89}  # quantize.py:214


def _qmax(num_bits):
    if num_bits is None or num_bits < 1 or num_bits > 8:
        raise ValueError(f"qnn: the int8 path supports 1..8-bit quantization, got num_bits={num_bits}")
    return float(2 ** num_bits - 1)


def _require_device(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"qnn: {what} runs on the MI355X int8 path only (ROCm device tensor required, got "
                           f"{t.device}); the reference's CPU fake-quant forward lives in oracle/ as a test checker")
    if t.dtype != torch.float32:
        raise TypeError(f"qnn: {what} expects float32 input, got {t.dtype}")


def float_scale(mn, mx, num_bits):
    """Scale of the Python-float path (quantize.py:71-75): double, floored at 1e-8.
    The kernels receive its fp32 rounding (the cast PyTorch applies at div_/mul_)."""
    return max((float(mx) - float(mn)) / (2.0 ** num_bits - 1.0), 1e-8)


def _round_up(a, b):
    return (a + b - 1) // b * b


# ============================================================ functional quantize
class _Passthrough(torch.autograd.Function):
    """A quantized value already computed on the device, with the straight-through gradient
    to the tensor it quantizes (quantize.py:105-109)."""

    @staticmethod
    def forward(ctx, x, q):
        return q.clone()  # a fresh tensor: a view of an input could not be modified in place downstream

    @staticmethod
    def backward(ctx, g):
        return g, None


class _QuantizeSTE(torch.autograd.Function):
    """UniformQuantize (quantize.py:39-109) under autograd: the device fake-quantizer
    forward, the straight-through estimator backward (:105-109)."""

    @staticmethod
    def forward(ctx, x, num_bits, min_value, max_value, num_chunks):
        return _quantize_fwd(x.detach(), num_bits, min_value, max_value, num_chunks)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None, None, None


def quantize(x, num_bits=8, min_value=None, max_value=None, num_chunks=None, stochastic=False, inplace=False):
    """quantize.py:159-160 with its effective binding: `stochastic` is never set and
    the asymmetric branch always runs.  GPU only.  Under autograd
    (training) the gradient passes straight through (:105-109)."""
    if torch.is_grad_enabled() and x.requires_grad:
        return _QuantizeSTE.apply(x, num_bits, min_value, max_value, num_chunks)
    return _quantize_fwd(x, num_bits, min_value, max_value, num_chunks, inplace)


def _quantize_fwd(x, num_bits=8, min_value=None, max_value=None, num_chunks=None, inplace=False):
    _require_device(x, "quantize()")
    qmax = _qmax(num_bits)
    xc = x.contiguous()
    out = xc if inplace else torch.empty_like(xc)
    st = _lib.stream_of(xc)
    if min_value is None or max_value is None:
        if (min_value is None) != (max_value is None):
            raise NotImplementedError("qnn: quantize() with only one of min/max given")
        B = x.shape[0]
        chunks = B if num_chunks is None else num_chunks
        if max(B // chunks, 1) != 1 or xc.numel() > 65536:
            raise NotImplementedError("qnn: per-chunk ranges are only used by training paths (out of scope)")
        _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(xc), _lib.ptr(out), xc.numel(), qmax, 0, None, st)
        return out
    if torch.is_tensor(min_value) or torch.is_tensor(max_value):
        mn = torch.as_tensor(min_value, dtype=torch.float32, device=x.device)
        mx = torch.as_tensor(max_value, dtype=torch.float32, device=x.device)
        rows = mn.numel()
        if rows == 1:
            mn, mx = mn.reshape(1), mx.reshape(1)
        elif mn.shape[0] != x.shape[0] or mn.numel() != x.shape[0]:
            raise NotImplementedError("qnn: tensor ranges must be per-tensor or per-dim-0")
        mn, mx = mn.contiguous(), mx.contiguous()
        _lib.call("qnn_fake_quant_rows_f32", _lib.ptr(xc), _lib.ptr(out), rows, xc.numel() // rows,
                  _lib.ptr(mn), _lib.ptr(mx), qmax, st)
        return out
    s = float_scale(min_value, max_value, num_bits)
    _lib.call("qnn_fake_quant_f32", _lib.ptr(xc), _lib.ptr(out), xc.numel(), -float(min_value), float(min_value),
              s, qmax, st)
    return out


def grad_noise(like):
    """The stochastic-rounding draw of the gradient quantizer: `output.new(output.shape)
    .uniform_(-0.5, 0.5)` (quantize.py:92-94), on the gradient's device.  Module-level so a
    test can substitute a fixed draw (GRAD_NOISE[0])."""
    return torch.empty_like(like).uniform_(-0.5, 0.5)


GRAD_NOISE = [grad_noise]


def quantize_grad_tensor(g, num_bits=8, min_value=None, max_value=None, stochastic=True):
    """UniformQuantizeGrad.backward (quantize.py:123-139) on a gradient tensor: the range
    from the gradient as Python floats, then UniformQuantize().apply(grad, num_bits, min, max,
    stochastic, inplace) -- which binds enforce_true_zero=True (:41-43), so the zero point is
    integral (:76-87) -- on the device (qnn_grad_quant_f32)."""
    _require_device(g, "quantize_grad")
    gc = g.contiguous()
    mn = float(gc.min()) if min_value is None else float(min_value)
    mx = float(gc.max()) if max_value is None else float(max_value)
    qmin, qmax = 0.0, 2.0 ** num_bits - 1.0
    scale = max((mx - mn) / (qmax - qmin), 1e-8)
    izp = qmin - mn / scale
    zp = int(qmin if izp < qmin else (qmax if izp > qmax else izp))
    noise = GRAD_NOISE[0](gc).contiguous() if stochastic else None
    out = torch.empty_like(gc)
    _lib.call("qnn_grad_quant_f32", _lib.ptr(gc), _lib.ptr(noise), _lib.ptr(out), gc.numel(),
              float(np.float32(scale)), float(zp), qmax, _lib.stream_of(gc))
    return out


class _QuantizeGrad(torch.autograd.Function):
    """UniformQuantizeGrad (quantize.py:112-139): identity forward, quantized gradient."""

    @staticmethod
    def forward(ctx, x, num_bits, min_value, max_value, stochastic):
        ctx.args = (num_bits, min_value, max_value, stochastic)
        # the reference returns its input (quantize.py:121); a copy here, because the models
        # apply nn.ReLU(inplace=True) to this output and autograd forbids in-place writes to a
        # view returned by a custom Function
        return x.clone()

    @staticmethod
    def backward(ctx, grad_output):
        return quantize_grad_tensor(grad_output, *ctx.args), None, None, None, None


def quantize_grad(x, num_bits=8, min_value=None, max_value=None, stochastic=True, inplace=False):
    """UniformQuantizeGrad (quantize.py:112-121, :163-164): identity in forward; under
    autograd the backward quantizes the incoming gradient (quantize_grad_tensor)."""
    if torch.is_grad_enabled() and x.requires_grad:
        return _QuantizeGrad.apply(x, num_bits, min_value, max_value, stochastic)
    return x


def conv2d_biprec(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, num_bits_grad=None):
    """quantize.py:142-148: out1 (input detached) carries the weight/bias gradient, out2
    (weight/bias detached) the input gradient through the gradient quantizer; the forward
    value out1 + out2 - out1 is one conv bitwise."""
    out1 = F.conv2d(input.detach(), weight, bias, stride, padding, dilation, groups)
    out2 = F.conv2d(input, weight.detach(), bias.detach() if bias is not None else None, stride, padding, dilation,
                    groups)
    out2 = quantize_grad(out2, num_bits=num_bits_grad)
    return out1 + out2 - out1.detach()


def linear_biprec(input, weight, bias=None, num_bits_grad=None):
    """quantize.py:151-156."""
    out1 = F.linear(input.detach(), weight, bias)
    out2 = F.linear(input, weight.detach(), bias.detach() if bias is not None else None)
    out2 = quantize_grad(out2, num_bits=num_bits_grad)
    return out1 + out2 - out1.detach()


class _QLayerTrain(torch.autograd.Function):
    """The training forward of QConv2d / QLinear (quantize.py:314-354, :398-432): the int8
    MFMA forward (bitwise the eval kernel's output for the same ranges), and the backward
    autograd derives from the reference's graph --
      input_  = quantize_input(input)          straight-through (:105-109)
      qweight = quantize(weight, w_min, w_max) straight-through
      qbias   = quantize(bias, b_min, b_max)   straight-through
      output  = F.conv2d(input_, qweight, qbias)                 [num_bits_grad None]
              = quantize_grad(F.conv2d(...))                     [num_bits_grad, no biprecision]
              = conv2d_biprec(...)                               [num_bits_grad and biprecision]
    so grad_input = conv_input(qweight, g_in), grad_weight = conv_weight(input_, g_w),
    grad_bias = sum(g_w), with g_in = g_w = the (possibly quantized) output gradient, except
    under biprecision where only g_in is quantized.  The transposed contractions are fp32
    (torch's conv backward); only the quantization semantics are this row's."""

    @staticmethod
    def forward(ctx, input, weight, bias, mod, rng, fwd):
        ctx.mod, ctx.rng = mod, rng
        ctx.save_for_backward(input, weight, bias)
        with torch.no_grad():
            return fwd(input.detach())

    @staticmethod
    def backward(ctx, gy):
        x, w, b = ctx.saved_tensors
        mod = ctx.mod
        gy = gy.contiguous()
        g_in = g_w = gy
        if mod.num_bits_grad is not None:
            gq = quantize_grad_tensor(gy, mod.num_bits_grad)
            g_in = gq
            if not mod.biprecision:
                g_w = gq
        with torch.no_grad():
            xh = _quantize_fwd(x.detach().contiguous(), mod.num_bits, ctx.rng[0], ctx.rng[1])
            wh = _quantize_fwd(w.detach().contiguous(), mod.num_bits_weight, mod.weight_min, mod.weight_max)
            gx = gw = gb = None
            if isinstance(mod, nn.Conv2d):
                args = (mod.stride, mod.padding, mod.dilation, mod.groups)
                if ctx.needs_input_grad[0]:
                    gx = torch.nn.grad.conv2d_input(x.shape, wh, g_in, *args)
                if ctx.needs_input_grad[1]:
                    gw = torch.nn.grad.conv2d_weight(xh, w.shape, g_w, *args)
                if b is not None and ctx.needs_input_grad[2]:
                    gb = g_w.sum((0, 2, 3))
            else:
                if ctx.needs_input_grad[0]:
                    gx = g_in @ wh
                if ctx.needs_input_grad[1]:
                    gw = g_w.reshape(-1, g_w.shape[-1]).t() @ xh.reshape(-1, xh.shape[-1])
                if b is not None and ctx.needs_input_grad[2]:
                    gb = g_w.reshape(-1, g_w.shape[-1]).sum(0)
        return gx, gw, gb, None, None, None


def _needs_grad(input, mod):
    return torch.is_grad_enabled() and (input.requires_grad or mod.weight.requires_grad or
                                        (mod.bias is not None and mod.bias.requires_grad))


# ============================================================ QuantNode / QuantMeasure
class QuantNode:
    """quantize.py:177-196."""

    def __init__(self):
        self.enable_quant = True
        self.freeze_param_dyn_range = False

    def set_measure_mode(self, measure, momentum=None):
        self.enable_quant = not measure
        if momentum and isinstance(self, QuantMeasure):
            self.momentum = momentum
        else:
            if isinstance(self, nn.Module):
                for q in self._modules.values():
                    if isinstance(q, QuantNode):
                        q.set_measure_mode(measure, momentum=momentum)

    def overwrite_params(self, logging=None):
        if isinstance(self, nn.Module):
            for q in self._modules.values():
                if isinstance(q, QuantNode):
                    q.overwrite_params(logging)


def measure_stats(x):
    """QuantMeasure's batch statistics (quantize.py:226-233) on the device: 0-dim fp32
    tensors (mean of per-sample min, mean of per-sample max, mean, unbiased std)."""
    _require_device(x, "QuantMeasure calibration")
    xc = x.detach().contiguous()
    B = xc.size(0)
    lib = _lib.load()
    work = torch.empty(lib.qnn_measure_stats_work(B), dtype=torch.float64, device=xc.device)
    out = torch.empty(4, dtype=torch.float32, device=xc.device)
    _lib.call("qnn_measure_stats_f32", _lib.ptr(xc), B, xc.numel() // B, _lib.ptr(work), _lib.ptr(out),
              _lib.stream_of(xc))
    return out[0], out[1], out[2], out[3]


def rangebn_stats(x, num_chunks):
    """RangeBN's train reductions (quantize.py:467-472) on the device: per-channel
    (mean of chunk maxima, mean of chunk minima, mean) and the chunk length."""
    _require_device(x, "RangeBN calibration")
    xc = x.detach().contiguous()
    B, C, H, W = xc.shape
    if (B * H * W) % num_chunks:
        raise ValueError(f"qnn: RangeBN statistics need B*H*W % num_chunks == 0 (got {B * H * W}, {num_chunks})")
    work = torch.empty(3 * C * num_chunks, dtype=torch.float64, device=xc.device)
    mm, mn, mean = (torch.empty(C, dtype=torch.float32, device=xc.device) for _ in range(3))
    _lib.call("qnn_rangebn_stats_f32", _lib.ptr(xc), B, C, H * W, num_chunks, _lib.ptr(work), _lib.ptr(mm),
              _lib.ptr(mn), _lib.ptr(mean), _lib.stream_of(xc))
    return mm, mn, mean, B * H * W // num_chunks


class QuantMeasure(nn.Module, QuantNode):
    """quantize.py:198-268: per-tensor activation range; eval = running range."""
    _QMEASURE_SUPPORTED_METHODS = ["avg", "aciq"]

    def __init__(self, num_bits=8, momentum=None, method="avg"):
        super().__init__()
        QuantNode.__init__(self)
        assert method in QuantMeasure._QMEASURE_SUPPORTED_METHODS
        self.register_buffer("running_min", torch.zeros(1))
        self.register_buffer("running_max", torch.zeros(1))
        self.register_buffer("num_measurements", torch.zeros(1))
        self.register_buffer("running_var", torch.ones(1))
        self.register_buffer("running_mean", torch.zeros(1))
        self.momentum = momentum
        self.num_bits = num_bits
        self.method = method
        self.laplace_alpha = _QMEASURE_ALPHA.get(num_bits)
        self._range_cache = None

    def _momentum_update_stat(self, new_value, running_stat, momentum=None):
        momentum = momentum or self.momentum or self.num_measurements / (self.num_measurements + 1)
        running_stat.mul_(momentum).add_(new_value * (1 - momentum))

    def _observe(self, input_):
        """Train-branch statistics (quantize.py:225-239); returns the batch range.  The
        reductions run in one device pass (qnn_measure_stats_f32); the momentum updates
        are the reference's torch ops."""
        min_value, max_value, mean, std = measure_stats(input_)
        self._momentum_update_stat(min_value, self.running_min)
        self._momentum_update_stat(max_value, self.running_max)
        self._momentum_update_stat(mean, self.running_mean)
        self._momentum_update_stat(std, self.running_var)
        self.num_measurements += 1
        if self.method == "aciq":
            min_value, max_value = self._get_aciq_range(std, mean, min_value, max_value)
        return float(min_value), float(max_value)

    def _eval_range(self):
        """(float min, float max) of the eval branch (:241-249), cached on buffer versions."""
        if self.method == "aciq":
            # `std += 1e-8` mutates running_var in place every call (:258): keep that.
            lo, hi = self._get_aciq_range(self.running_var, self.running_mean, self.running_min, self.running_max)
            return float(lo), float(hi)
        key = (self.running_min.data_ptr(), self.running_min._version,
               self.running_max.data_ptr(), self.running_max._version)
        if self._range_cache is None or self._range_cache[0] != key:
            self._range_cache = (key, (float(self.running_min), float(self.running_max)))
        return self._range_cache[1]

    def range_for(self, input):
        """The (min, max) the forward quantizes `input` with, applying the
        training-branch side effects exactly when the reference does."""
        if self.training:
            with torch.no_grad():
                return self._observe(input.detach())
        return self._eval_range()

    def forward(self, input):
        rng = self.range_for(input)
        if self.enable_quant:
            return quantize(input, self.num_bits, min_value=rng[0], max_value=rng[1])
        return input

    def _get_measured_range(self):
        return float(self.running_min), float(self.running_max)

    def _get_aciq_range(self, std, mean, tmin, tmax):
        with torch.no_grad():
            std += 1e-8
            assert self.laplace_alpha, "aciq not supported for module num bits"
            clip_val = std * self.laplace_alpha
            assert clip_val > 0, "invalid clip value!"
            max_range = tmax - tmin
            clip_val = min(max_range / 2, clip_val)
            min_value = max(tmin, mean - clip_val)
            max_value = min(tmax, mean + clip_val)
        return min_value, max_value


# ============================================================ packed operands
class _Packed:
    """Device-resident int8 operands of one QConv2d/QLinear weight version."""
    __slots__ = ("key", "wq", "s_w", "b_w", "tap_sum", "w_hat", "qbias", "cin_pad", "cout_pad", "kpad", "s2d",
                 "ptaps", "kmask", "geom", "epi")


def border_classes(size, k, stride, pad, out):
    """Distinct [lo, hi) valid-tap ranges over the output positions of one spatial
    dim (zero padding): the classes of the border-aware zero-point table."""
    cls, ranges, ids = [], [], {}
    for o in range(out):
        lo = max(0, pad - o * stride)
        hi = min(k, size + pad - o * stride)
        key = (lo, hi)
        if key not in ids:
            ids[key] = len(ranges)
            ranges.append(key)
        cls.append(ids[key])
    return cls, ranges


def channel_pad(c):
    """Cp = 16 * 2^j >= c (the kernel's K-chunk addressing needs a power of two)."""
    cp = 16
    while cp < c:
        cp *= 2
    return cp


def use_s2d(cin_g, kh, stride):
    """Space-to-depth for stride-2 stems on <= 4 channels (7x7/2, 3x3/2)."""
    return tuple(stride) == (2, 2) and 4 * cin_g <= 16 and kh > 1


def s2d_kmask(kh, kw, cin_g, kpad, dev):
    """K-mask of a space-to-depth packed row: 1 where byte (tap (a,b), channel (2u+v)*cin+ci)
    is a real kernel tap (2a+u < kh, 2b+v < kw), else 0 (include/qnn.h, qnn_conv_desc.kmask)."""
    pkw = (kw + 1) // 2
    m = np.zeros(kpad, dtype=np.int8)
    for a in range((kh + 1) // 2):
        for b in range(pkw):
            for uv in range(4):
                u, v = uv >> 1, uv & 1
                if 2 * a + u < kh and 2 * b + v < kw:
                    base = (a * pkw + b) * 16 + uv * cin_g
                    m[base:base + cin_g] = 1
    return torch.from_numpy(m).to(dev)


# QNN_MODULE_AUTOTUNE=1 (or MODULE_AUTOTUNE[0] = True): the drop-in module path times every tile
# configuration of a layer the first time it sees an input shape and keeps the fastest; off, it
# launches the library's cost-model choice.
MODULE_AUTOTUNE = [os.environ.get("QNN_MODULE_AUTOTUNE", "0") == "1"]

# QNN_FUSED_INPUT=1 (or FUSED_INPUT[0] = True; per layer: qnn_fused_input = True / False): a drop-in
# 3x3 conv on 64 or 128 input channels quantizes its fp32 input inside the convolution
# (qnn_qconv2d_fwd_nchw_f32, one launch) instead of a quantize launch + the conv.  Bitwise the same
# output either way; DESIGN.md records the measured trade (profiles/r5_bench_layers_dropin.jsonl).
FUSED_INPUT = [os.environ.get("QNN_FUSED_INPUT", "0") == "1"]


class _QLayerMixin:
    """Shared int8 machinery of QConv2d / QLinear (QuantNode subclasses)."""

    def _init_qcache(self):
        self._qpack = None
        # qnn_conv_desc.tile of the int8 contraction: 0 = the library's cost model, k + 1 =
        # configuration k (qnn_conv_plan); every configuration computes the identical result
        self.qnn_tile = 0
        self.qnn_keep_input = False
        self.qnn_fused_input = None  # None: FUSED_INPUT[0]
        self.qnn_fused_tile = 0      # its configuration: 0 = the cheapest that fits, k + 1 = k
        self._last_fused = False     # whether the last forward took the one-launch path

    def _weight4(self):
        w = self.weight
        return w if w.dim() == 4 else w.view(w.shape[0], w.shape[1], 1, 1)

    def _pack(self, depthwise=False, s2d=False):
        w = self.weight
        bias = self.bias
        freeze = bool(self.freeze_param_dyn_range)
        frozen = None
        if freeze:  # the frozen range buffers feed the quantizers: their versions key the pack too
            frozen = tuple((t.data_ptr(), t._version) for t in (self.weight_min, self.weight_max,
                                                                  getattr(self, "bias_min", None),
                                                                  getattr(self, "bias_max", None))
                           if torch.is_tensor(t))
        key = (w.data_ptr(), w._version, None if bias is None else (bias.data_ptr(), bias._version), freeze, frozen,
               self.num_bits_weight, self.bias_quant, depthwise, s2d, w.device)
        pk = self._qpack
        if pk is not None and pk.key == key:
            return pk
        if not self.per_channel:
            # the reference assigns a float to a registered buffer here and raises (quantize.py:325-326)
            raise TypeError("cannot assign 'float' as buffer 'weight_min' (torch.Tensor or None expected)")
        _require_device(w, type(self).__name__)
        qmax = _qmax(self.num_bits_weight)
        w4 = self._weight4().detach().contiguous()
        cout, cin_g, kh, kw = w4.shape
        dev = w.device
        pk = _Packed()
        pk.key = key
        pk.s2d = s2d
        if s2d:
            pk.cin_pad = 16
            pk.ptaps = ((kh + 1) // 2) * ((kw + 1) // 2)
        else:
            pk.cin_pad = channel_pad(cin_g)
            pk.ptaps = kh * kw
        pk.cout_pad = _round_up(cout, 64) if cout <= 64 else _round_up(cout, 128)
        pk.kpad = _round_up(pk.ptaps * pk.cin_pad, 128)
        pk.kmask = s2d_kmask(kh, kw, cin_g, pk.kpad, dev) if s2d else None
        pk.wq = torch.empty((pk.cout_pad, pk.kpad), dtype=torch.int8, device=dev)
        pk.s_w = torch.empty(cout, dtype=torch.float32, device=dev)
        pk.b_w = torch.empty(cout, dtype=torch.float32, device=dev)
        pk.tap_sum = torch.empty((cout, kh * kw), dtype=torch.float32, device=dev)
        pk.w_hat = torch.empty((cout, cin_g * kh * kw), dtype=torch.float32, device=dev) if depthwise else None
        st = _lib.stream_of(w4)
        if freeze:
            wmin_in = self.weight_min.detach().reshape(-1).float().contiguous()
            wmax_in = self.weight_max.detach().reshape(-1).float().contiguous()
            wmin_out = wmax_out = None
        else:
            wmin_in = wmax_in = None
            # weight_min/max buffers are rewritten every forward (quantize.py:317-323)
            wmin_out = torch.empty(cout, dtype=torch.float32, device=dev)
            wmax_out = torch.empty(cout, dtype=torch.float32, device=dev)
        _lib.call("qnn_pack_weight_i8", _lib.ptr(w4), cout, cin_g, kh, kw, pk.cin_pad, pk.cout_pad, 2 if s2d else 0,
                  qmax, _lib.ptr(wmin_in), _lib.ptr(wmax_in), _lib.ptr(pk.wq), _lib.ptr(pk.s_w), _lib.ptr(pk.b_w),
                  _lib.ptr(pk.tap_sum), _lib.ptr(pk.w_hat), _lib.ptr(wmin_out), _lib.ptr(wmax_out), st)
        if not freeze:
            self.weight_min = wmin_out.view(self.scale_shape)
            self.weight_max = wmax_out.view(self.scale_shape)
        pk.qbias = None
        if bias is not None:
            b = bias.detach().contiguous()
            rng = torch.empty(2, dtype=torch.float32, device=dev)
            if self.bias_quant and freeze:
                # frozen: quantize(bias, min_value=self.bias_min, max_value=self.bias_max) (quantize.py:336-338)
                pk.qbias = torch.empty_like(b)
                bmin = self.bias_min.detach().reshape(1).float().contiguous()
                bmax = self.bias_max.detach().reshape(1).float().contiguous()
                _lib.call("qnn_fake_quant_rows_f32", _lib.ptr(b), _lib.ptr(pk.qbias), 1, b.numel(), _lib.ptr(bmin),
                          _lib.ptr(bmax), qmax, st)
            elif self.bias_quant:
                pk.qbias = torch.empty_like(b)
                _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(b), _lib.ptr(pk.qbias), b.numel(), qmax, 0,
                          _lib.ptr(rng), st)
            else:
                pk.qbias = b
                tmp = torch.empty_like(b)
                _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(b), _lib.ptr(tmp), b.numel(), qmax, 0, _lib.ptr(rng), st)
            if not freeze:
                # quantize.py:328-330 (tensor assignment, also when bias_quant is off)
                self.bias_min = rng[0]
                self.bias_max = rng[1]
        pk.geom = {}
        pk.epi = {}
        self._qpack = pk
        return pk

    def _tuned_tile(self, xq, pk, d, e, st, key, reps=3):
        """The fastest tile configuration for this layer at this input shape, timed once on the
        device (HIP events on the launch stream) the first time the shape is seen, as the
        engine's autotune does; every configuration computes the identical output, so this
        only changes speed.  0 (the cost model) while a hipGraph is being captured."""
        tuned = self.__dict__.setdefault("_tuned", {})
        if key in tuned:
            return tuned[key]
        best = None
        for k in range(_lib.CONV_TILES):
            d.tile = k + 1
            try:
                _lib.call("qnn_qconv2d_fwd", _lib.ptr(xq), _lib.ptr(pk.wq), ctypes.byref(d), ctypes.byref(e), st)
            except _lib.QnnError:
                continue  # configuration not built for this layer
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                _lib.call("qnn_qconv2d_fwd", _lib.ptr(xq), _lib.ptr(pk.wq), ctypes.byref(d), ctypes.byref(e), st)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / reps
            if best is None or ms < best[1]:
                best = (k, ms)
        tuned[key] = 0 if best is None else best[0] + 1
        return tuned[key]

    @staticmethod
    def _geometry(pk, H, W, kh, kw, sh, sw, ph, pw, Ho, Wo, dev):
        gk = (H, W)
        g = pk.geom.get(gk)
        if g is None:
            hc, hr = border_classes(H, kh, sh, ph, Ho)
            wc, wr = border_classes(W, kw, sw, pw, Wo)
            if len(hr) * len(wr) > 64:
                raise NotImplementedError("qnn: more than 64 border classes")
            t = lambda a: torch.tensor(np.asarray(a, dtype=np.int32).reshape(-1), device=dev)
            g = (t(hc), t(hr), len(hr), t(wc), t(wr), len(wr))
            pk.geom[gk] = g
        return g

    @staticmethod
    def _epilogue(pk, g, gk, s_x, b_x, kh, kw):
        ek = (gk, s_x, b_x)
        e = pk.epi.get(ek)
        if e is None:
            hcls, hr, nhc, wcls, wr, nwc = g
            cout = pk.s_w.numel()
            sxsw = (pk.s_w.double() * float(s_x)).float()
            sxbw = (pk.b_w.double() * float(s_x)).float()
            table = torch.empty((nhc, nwc, cout), dtype=torch.float32, device=pk.s_w.device)
            _lib.call("qnn_conv_border_table", _lib.ptr(pk.tap_sum), cout, kh, kw, _lib.ptr(hr), nhc, _lib.ptr(wr),
                      nwc, float(b_x), _lib.ptr(table), _lib.stream_of(table))
            e = (sxsw, sxbw, table)
            if len(pk.epi) > 8:
                pk.epi.clear()
            pk.epi[ek] = e
        return e

    def _int8_forward(self, x4, rng, stride, padding):
        """Quantize x (NCHW fp32) into the padded (or space-to-depth) NHWC8 layout and
        run the MFMA conv in drop-in mode (fp32 NCHW out)."""
        w4 = self._weight4()
        cout, cin_g, kh, kw = w4.shape
        N, C, H, W = x4.shape
        if C != cin_g:
            raise RuntimeError(f"qnn: expected {cin_g} input channels, got {C}")
        sh, sw = stride
        ph, pw = padding
        if ph != pw:
            raise NotImplementedError("qnn: asymmetric padding is not on the int8 path")
        s2d = use_s2d(cin_g, kh, stride)
        pk = self._pack(s2d=s2d)
        Ho = (H + 2 * ph - kh) // sh + 1
        Wo = (W + 2 * pw - kw) // sw + 1
        if Ho <= 0 or Wo <= 0:
            raise RuntimeError("qnn: output size is empty")
        qmax = _qmax(self.num_bits)
        mn, mx = rng
        s = float_scale(mn, mx, self.num_bits)
        s32 = float(np.float32(s))
        b_x = 128.0 * s32 + float(np.float32(mn))
        dev = x4.device
        st = _lib.stream_of(x4)
        d = _lib.ConvDesc()
        d.n, d.cout, d.cout_pad, d.ho, d.wo, d.kpad = N, cout, pk.cout_pad, Ho, Wo, pk.kpad
        if s2d:
            d.kh, d.kw, d.sh, d.sw, d.cp = (kh + 1) // 2, (kw + 1) // 2, 1, 1, 16
            d.hp, d.wp = Ho - 1 + d.kh, Wo - 1 + d.kw
            nbytes = N * d.hp * d.wp * 16
            xq = torch.empty(nbytes + 128, dtype=torch.int8, device=dev)
            _lib.call("qnn_quantize_nchw_to_s2d8", _lib.ptr(x4), _lib.ptr(xq), N, C, H, W, ph, d.hp, d.wp, -float(mn),
                      s, qmax, st)
        else:
            d.kh, d.kw, d.sh, d.sw, d.cp = kh, kw, sh, sw, pk.cin_pad
            d.hp, d.wp = H + 2 * ph, W + 2 * pw
            nbytes = N * d.hp * d.wp * d.cp
            xq = None
        d.zero_off = nbytes
        d.kmask = None if pk.kmask is None else pk.kmask.data_ptr()
        d.tile = int(self.qnn_tile)
        g = self._geometry(pk, H, W, kh, kw, sh, sw, ph, pw, Ho, Wo, dev)
        sxsw, sxbw, table = self._epilogue(pk, g, (H, W), s32, b_x, kh, kw)
        y = torch.empty((N, cout, Ho, Wo), dtype=torch.float32, device=dev)
        e = _lib.Epilogue()
        e.mode = 0
        e.sxsw, e.sxbw, e.table, e.hcls, e.wcls = (sxsw.data_ptr(), sxbw.data_ptr(), table.data_ptr(),
                                                   g[0].data_ptr(), g[3].data_ptr())
        e.nwc, e.nclass = g[5], g[2] * g[5]
        e.bias = None if pk.qbias is None else pk.qbias.data_ptr()
        e.out_f32 = y.data_ptr()
        if xq is None:
            fused = self.qnn_fused_input if self.qnn_fused_input is not None else FUSED_INPUT[0]
            # quantize-on-load: one launch reads the fp32 input (qnn_qconv2d_fwd_nchw_f32), when a
            # persistent-band configuration fits the layer; else quantize, then convolve
            if fused and pk.kmask is None and x4.is_contiguous() and _lib.call_unsupported_ok(
                    "qnn_qconv2d_fwd_nchw_f32", _lib.ptr(x4), C, H, W, ph, -float(mn), s, qmax, _lib.ptr(pk.wq),
                    ctypes.byref(d), ctypes.byref(e), int(self.qnn_fused_tile), st):
                self._last_conv = (d, e)
                self._last_xq = None
                self._last_fused = True
                return y
            xq = torch.empty(nbytes + 128, dtype=torch.int8, device=dev)
            _lib.call("qnn_quantize_nchw_to_nhwc8", _lib.ptr(x4), _lib.ptr(xq), N, C, H, W, ph, d.cp, -float(mn), s,
                      qmax, st)
        if self.qnn_tile == 0 and MODULE_AUTOTUNE[0] and not torch.cuda.is_current_stream_capturing():
            d.tile = self._tuned_tile(xq, pk, d, e, st, (N, H, W, Ho, Wo))
        _lib.call("qnn_qconv2d_fwd", _lib.ptr(xq), _lib.ptr(pk.wq), ctypes.byref(d), ctypes.byref(e), st)
        self._last_fused = False
        self._last_conv = (d, e)  # launch descriptors, for profiling tools (qnn_conv_plan)
        self._last_xq = xq if self.qnn_keep_input else None  # the codes, for tools that re-issue the launch
        return y


# ============================================================ QConv2d
class QConv2d(nn.Conv2d, QuantNode, _QLayerMixin):
    """quantize.py:271-354."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 num_bits=8, num_bits_weight=None, num_bits_grad=None, biprecision=False, bias_quant=True,
                 per_channel=True, **kwargs):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias, **kwargs)
        QuantNode.__init__(self)
        self._init_qcache()
        self.num_bits = num_bits
        self.num_bits_weight = num_bits_weight or num_bits
        self.num_bits_grad = num_bits_grad
        self.quantize_input = QuantMeasure(self.num_bits)
        self.biprecision = biprecision
        self.bias_quant = bias_quant and bias
        self.per_channel = per_channel
        if self.per_channel:
            n_channels = self.weight.size(0)
            dim = self.weight.dim()
            self.scale_shape = (n_channels,) + (1,) * (dim - 1)
            self.register_buffer("weight_min", self.weight.flatten(1).min(-1)[0].view(self.scale_shape))
            self.register_buffer("weight_max", self.weight.flatten(1).max(-1)[0].view(self.scale_shape))
        else:
            self.register_buffer("weight_min", self.weight.min())
            self.register_buffer("weight_max", self.weight.max())
        if self.bias_quant:
            self.register_buffer("bias_min", self.bias.min())
            self.register_buffer("bias_max", self.bias.max())

    def overwrite_params(self, logging=None):
        """quantize.py:301-312: bake the fake-quantized weight (and bias) into the state_dict."""
        sd = self.state_dict()
        if logging:
            logging.debug(f"quantizing parameters for {super().__str__()}")
        with torch.no_grad():
            sd.update({"weight": quantize(self.weight, num_bits=self.num_bits_weight, min_value=self.weight_min,
                                          max_value=self.weight_max)})
            if self.bias_quant:
                sd.update({"bias": quantize(self.bias, min_value=self.bias_min, max_value=self.bias_max,
                                            num_bits=self.num_bits_weight)})
        self.load_state_dict(sd)

    def _is_depthwise(self):
        return self.groups > 1 and self.groups == self.in_channels == self.out_channels

    def forward(self, input):
        rng = self.quantize_input.range_for(input)
        if not self.enable_quant:
            return F.conv2d(input, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        _require_device(input, "QConv2d")
        # the reference calls F.conv2d(input_, qweight, qbias, stride, padding, dilation, groups)
        # (quantize.py:342-344): padding_mode is never applied (zeros), string padding is F.conv2d's
        generic = (tuple(self.dilation) != (1, 1) or isinstance(self.padding, str) or
                   self.padding[0] != self.padding[1] or (self.groups != 1 and not self._is_depthwise()))

        def fwd(x):
            x = x.contiguous()
            if generic:
                return self._generic_forward(x, rng)
            if self._is_depthwise():
                return self._dw_forward(x, rng)
            return self._int8_forward(x, rng, self.stride, self.padding)

        if _needs_grad(input, self):  # training (§8(f4)): the same forward, the reference's backward
            return _QLayerTrain.apply(input, self.weight, self.bias, self, rng, fwd)
        with torch.no_grad():
            return fwd(input.detach())

    def _generic_forward(self, x, rng):
        """Dilated, grouped (other than depthwise) or unevenly / 'same'-padded QConv2d: the
        generic device conv (qnn_qconv2d_generic_fwd) on the fake-quantized operands."""
        pk = self._pack(depthwise=True)  # (its w_hat: the fake-quantized weight, any cin_g)
        N, C, H, W = x.shape
        cout, cin_g, kh, kw = self._weight4().shape
        if C != cin_g * self.groups:
            raise RuntimeError(f"qnn: expected {cin_g * self.groups} input channels, got {C}")
        sh, sw = self.stride
        dh, dw = self.dilation
        if isinstance(self.padding, str):
            if self.padding == "valid":
                pt = pb = pl = pr = 0
            else:  # 'same' (stride 1): F.conv2d puts the odd extra row / column at the bottom / right
                if (sh, sw) != (1, 1):
                    raise ValueError("padding='same' is not supported for strided convolutions")
                th, tw = dh * (kh - 1), dw * (kw - 1)
                pt, pl = th // 2, tw // 2
                pb, pr = th - pt, tw - pl
        else:
            pt = pb = self.padding[0]
            pl = pr = self.padding[1]
        Ho = (H + pt + pb - dh * (kh - 1) - 1) // sh + 1
        Wo = (W + pl + pr - dw * (kw - 1) - 1) // sw + 1
        if Ho <= 0 or Wo <= 0:
            raise RuntimeError("qnn: output size is empty")
        mn, mx = rng
        s = float_scale(mn, mx, self.num_bits)
        y = torch.empty((N, cout, Ho, Wo), dtype=torch.float32, device=x.device)
        _lib.call("qnn_qconv2d_generic_fwd", _lib.ptr(x), N, C, H, W, -float(mn), float(mn), s, _qmax(self.num_bits),
                  _lib.ptr(pk.w_hat), cout, self.groups, kh, kw, sh, sw, pt, pl, dh, dw, Ho, Wo, _lib.ptr(pk.qbias),
                  _lib.ptr(y), _lib.stream_of(x))
        return y

    def _dw_forward(self, x, rng):
        pk = self._pack(depthwise=True)
        N, C, H, W = x.shape
        kh, kw = self.kernel_size
        sh, sw = self.stride
        ph, pw = self.padding
        Ho = (H + 2 * ph - kh) // sh + 1
        Wo = (W + 2 * pw - kw) // sw + 1
        mn, mx = rng
        s = float_scale(mn, mx, self.num_bits)
        y = torch.empty((N, C, Ho, Wo), dtype=torch.float32, device=x.device)
        _lib.call("qnn_dwconv2d_fwd", _lib.ptr(x), N, C, H, W, _lib.ptr(pk.w_hat), kh, kw, sh, sw, ph, pw, Ho, Wo,
                  -float(mn), float(mn), s, _qmax(self.num_bits), _lib.ptr(pk.qbias), _lib.ptr(y), _lib.stream_of(x))
        return y


# ============================================================ QLinear
class QLinear(nn.Linear, QuantNode, _QLayerMixin):
    """quantize.py:357-432."""

    def __init__(self, in_features, out_features, bias=True, num_bits=8, num_bits_weight=None, num_bits_grad=None,
                 biprecision=False, bias_quant=True, per_channel=True, **kwargs):
        super().__init__(in_features, out_features, bias, **kwargs)
        QuantNode.__init__(self)
        self._init_qcache()
        self.num_bits = num_bits
        self.num_bits_weight = num_bits_weight or num_bits
        self.num_bits_grad = num_bits_grad
        self.biprecision = biprecision
        self.quantize_input = QuantMeasure(self.num_bits)
        self.bias_quant = bias_quant and bias
        self.per_channel = per_channel
        if self.per_channel:
            n_channels = self.weight.size(0)
            dim = self.weight.dim()
            self.scale_shape = (n_channels,) + (1,) * (dim - 1)
            self.register_buffer("weight_min", self.weight.flatten(1).min(-1)[0].view(self.scale_shape))
            self.register_buffer("weight_max", self.weight.flatten(1).max(-1)[0].view(self.scale_shape))
        else:
            self.register_buffer("weight_min", self.weight.min())
            self.register_buffer("weight_max", self.weight.max())
        if self.bias_quant:
            self.register_buffer("bias_min", self.bias.min())
            self.register_buffer("bias_max", self.bias.max())

    def overwrite_params(self, logging=None):
        """quantize.py:386-396."""
        sd = self.state_dict()
        if logging:
            logging.debug(f"quantizing parameters for {super().__str__()}")
        with torch.no_grad():
            sd.update({"weight": quantize(self.weight, num_bits=self.num_bits_weight, min_value=self.weight_min,
                                          max_value=self.weight_max)})
            if self.bias_quant:
                sd.update({"bias": quantize(self.bias, min_value=self.bias_min, max_value=self.bias_max,
                                            num_bits=self.num_bits_weight)})
        self.load_state_dict(sd)

    def forward(self, input):
        rng = self.quantize_input.range_for(input)
        if not self.enable_quant:
            return F.linear(input, self.weight, self.bias)
        _require_device(input, "QLinear")
        lead = input.shape[:-1]

        def fwd(x):
            x = x.reshape(-1, input.shape[-1]).contiguous()
            y = self._int8_forward(x.view(x.shape[0], x.shape[1], 1, 1), rng, (1, 1), (0, 0))
            return y.view(*lead, self.out_features)

        if _needs_grad(input, self):  # training (§8(f4))
            return _QLayerTrain.apply(input, self.weight, self.bias, self, rng, fwd)
        with torch.no_grad():
            return fwd(input.detach())


# ============================================================ RangeBN
class RangeBN(nn.Module):
    """quantize.py:435-505 (normalized RangeBN).  Eval on a ROCm device runs one
    fused HIP kernel; train (calibration) keeps the reference's torch-op statistics."""

    def __init__(self, num_features, dim=1, momentum=0.1, affine=True, num_chunks=16, eps=1e-5, num_bits=8,
                 num_bits_grad=8):
        super().__init__()
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.zeros(num_features))
        self.momentum = momentum
        self.dim = dim
        if affine:
            self.bias = nn.Parameter(torch.Tensor(num_features))
            self.weight = nn.Parameter(torch.Tensor(num_features))
        else:
            self.register_parameter("bias", None)
            self.register_parameter("weight", None)
        self.num_bits = num_bits
        self.num_bits_grad = num_bits_grad
        self.quantize_input = QuantMeasure(self.num_bits)
        self.eps = eps
        self.num_chunks = num_chunks
        self._pcache = None
        self.reset_params()

    def reset_params(self):
        if self.weight is not None:
            self.weight.data.uniform_()
        if self.bias is not None:
            self.bias.data.zero_()

    def _params(self, scale):
        """Fake-quantized (scale, weight, bias) vectors (:486-499), cached on versions."""
        w, b = self.weight, self.bias
        key = (scale.data_ptr(), scale._version, None if w is None else (w.data_ptr(), w._version),
               None if b is None else (b.data_ptr(), b._version), self.num_bits)
        if self._pcache is not None and self._pcache[0] == key:
            return self._pcache[1]
        qmax = _qmax(self.num_bits)
        st = _lib.stream_of(scale)
        C = scale.numel()
        sq = torch.empty(C, dtype=torch.float32, device=scale.device)
        _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(scale.contiguous()), _lib.ptr(sq), C, qmax, 1, None, st)
        if w is not None:
            wq = torch.empty_like(sq)
            _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(w.detach().contiguous()), _lib.ptr(wq), C, qmax, 1, None, st)
        else:
            wq = torch.ones_like(sq)
        if b is not None:
            bq = torch.empty_like(sq)
            _lib.call("qnn_fake_quant_vec_f32", _lib.ptr(b.detach().contiguous()), _lib.ptr(bq), C, qmax, 0, None, st)
        else:
            bq = torch.zeros_like(sq)
        out = (sq, wq, bq)
        self._pcache = (key, out)
        return out

    def forward(self, x):
        if self.training or not self.quantize_input.enable_quant:
            return self._forward_reference_ops(x)
        _require_device(x, "RangeBN")
        squeeze = x.dim() == 2
        x4 = x.unsqueeze(-1).unsqueeze(-1) if squeeze else x
        x4 = x4.detach().contiguous()
        rng = self.quantize_input.range_for(x4)
        mn, mx = rng
        s = float_scale(mn, mx, self.num_bits)
        N, C, H, W = x4.shape
        with torch.no_grad():
            sq, wq, bq = self._params(self.running_var)
            y = torch.empty_like(x4)
            _lib.call("qnn_rangebn_f32", _lib.ptr(x4), _lib.ptr(y), N, C, H * W, -float(mn), float(mn), s,
                      _qmax(self.num_bits), _lib.ptr(self.running_mean), _lib.ptr(sq), _lib.ptr(wq), _lib.ptr(bq),
                      None, 0, _lib.stream_of(x4))
        if y.size(3) == 1 and y.size(2) == 1:
            y = y.squeeze(-1).squeeze(-1)
        return y

    def _forward_reference_ops(self, x):
        """Train / measure-mode branch with torch ops (quantize.py:461-505)."""
        grad = torch.is_grad_enabled() and (x.requires_grad or any(
            p is not None and p.requires_grad for p in (self.weight, self.bias)))
        x = self.quantize_input(x)
        if x.dim() == 2:
            x = x.unsqueeze(-1).unsqueeze(-1)
        if self.training:
            if grad:  # training (§8(f4)): the statistics as the reference's differentiable torch ops
                B, C, H, W = x.shape
                y = x.transpose(0, 1).contiguous().view(C, self.num_chunks, B * H * W // self.num_chunks)
                mean_max = y.max(-1)[0].mean(-1)
                mean_min = y.min(-1)[0].mean(-1)
                mean = y.view(C, -1).mean(-1)
                n = y.size(-1)
            else:
                # calibration: the chunked reductions in one device pass (qnn_rangebn_stats_f32)
                mean_max, mean_min, mean, n = rangebn_stats(x, self.num_chunks)
            scale_fix = (0.5 * 0.35) * (1 + (math.pi * math.log(4)) ** 0.5) / ((2 * math.log(n)) ** 0.5)
            scale = 1 / ((mean_max - mean_min) * scale_fix + self.eps)
            self.running_mean.detach().mul_(self.momentum).add_(mean * (1 - self.momentum))
            self.running_var.detach().mul_(self.momentum).add_(scale * (1 - self.momentum))
        else:
            mean = self.running_mean
            scale = self.running_var
        with torch.no_grad():
            sq, wq, bq = self._params(scale.detach().contiguous()) if x.is_cuda else _cpu_unsupported("RangeBN")
        if grad:  # the quantizers of :486-498 are straight-through (:105-109)
            sq = _Passthrough.apply(scale, sq)
            if self.weight is not None:
                wq = _Passthrough.apply(self.weight, wq)
            if self.bias is not None:
                bq = _Passthrough.apply(self.bias, bq)
        out = (x - mean.view(1, mean.size(0), 1, 1)) * sq.view(1, sq.size(0), 1, 1)
        out = out * wq.view(1, wq.size(0), 1, 1)
        out = out + bq.view(1, bq.size(0), 1, 1)
        if grad and self.num_bits_grad is not None:
            out = quantize_grad(out, num_bits=self.num_bits_grad)  # :500-501
        if out.size(3) == 1 and out.size(2) == 1:
            out = out.squeeze(-1).squeeze(-1)
        return out


def _cpu_unsupported(what):
    raise RuntimeError(f"qnn: {what} needs a ROCm device (the CPU fake-quant reference lives in oracle/)")


# ============================================================ tree helpers (:508-610)
# (the training-only helpers set_bn_is_train / distill_set_train, quantize.py:523-545,
# :595-599, belong to the distillation trainer and are out of scope: SURVEY.md §2 row 10)
def is_bn(m):
    return isinstance(m, nn.BatchNorm2d) or isinstance(m, nn.BatchNorm1d)


def is_quant(m):
    return isinstance(m, QuantNode) or isinstance(m, QLinear) or isinstance(m, QConv2d)


def recursive_apply(model, func, *args):
    for m in model.children():
        func(m, *args)
        recursive_apply(m, func, *args)


def set_measure_mode(model, measure, momentum=None, logger=None):
    def func(m, *args):
        if is_bn(m):
            m.train(not measure)
        elif is_quant(m):
            m.set_measure_mode(measure, momentum=momentum)

    recursive_apply(model, func)


def set_quant_mode(model, quant, logger=None):
    def func(m, *args):
        if is_quant(m):
            m.enable_quant = quant

    recursive_apply(model, func)


def overwrite_params(model, logger=None):
    def func(m, *args):
        if is_quant(m):
            m.overwrite_params(logger)

    recursive_apply(model, func)


def freeze_quant_params(model, freeze=True, include_param_dyn_range=True, momentum="same", logger=None):
    """quantize.py:579-592.  Note: the reference sets `freeze_param_dyn_rang` (sic,
    :590), so the weight range is never actually frozen; mirrored for parity."""

    def func(m, *args):
        if isinstance(m, QuantMeasure):
            m.train(not freeze)
            if momentum != "same":
                m.momentum = momentum
        if include_param_dyn_range and isinstance(m, QuantNode):
            m.freeze_param_dyn_rang = freeze

    recursive_apply(model, func)


def set_global_quantization_method(model, method="aciq", logger=None):
    assert method in QuantMeasure._QMEASURE_SUPPORTED_METHODS

    def func(m, *args):
        if isinstance(m, QuantMeasure):
            m.method = method

    recursive_apply(model, func)
