"""ctypes binding of libqnn_hip.so (the C ABI declared in include/qnn.h).

The library is built in-tree (`make -C quantized.pytorch_amd`) and loaded from
this directory only.  There is no fallback: if it is missing, every quantized
op on a ROCm device raises `QnnLibraryError`.

torch must be imported before the library is loaded so that its HIP runtime
(SONAME libamdhip64.so.7) is the one the library binds to; streams and device
pointers are then shared with PyTorch.
"""
import ctypes
import os

import torch  # noqa: F401  (binds the process HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QNN_LIB") or os.path.join(_HERE, "libqnn_hip.so")  # QNN_LIB: diagnostic builds

ABI_VERSION = 9
CONV_TILES = 64  # tile configurations of qnn_qconv2d_fwd (qnn_conv_desc.tile = k + 1); == qnn_conv_tile_count()

c_int, c_i64, c_float, c_ptr = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p


class ConvDesc(ctypes.Structure):
    """qnn_conv_desc (include/qnn.h)."""
    _fields_ = [(n, c_int) for n in ("n", "hp", "wp", "cp", "zero_off", "cout", "cout_pad", "kh", "kw", "sh", "sw",
                                     "ho", "wo", "kpad")] + [("kmask", c_ptr), ("tile", c_int)]


class ResLink(ctypes.Structure):
    """qnn_res_link (include/qnn.h)."""
    _fields_ = [("code", c_ptr), ("mean", c_ptr), ("sq", c_ptr), ("wq", c_ptr), ("bq", c_ptr), ("min", c_float),
                ("scale", c_float)]


MAX_RES = 4  # QNN_MAX_RES
COMM_ID_BYTES = 128  # QNN_COMM_ID_BYTES


class Epilogue(ctypes.Structure):
    """qnn_epilogue (include/qnn.h)."""
    _fields_ = [("mode", c_int), ("sxsw", c_ptr), ("sxbw", c_ptr), ("table", c_ptr), ("hcls", c_ptr),
                ("wcls", c_ptr), ("nwc", c_int), ("nclass", c_int), ("bias", c_ptr),
                ("bn_mean", c_ptr), ("bn_sq", c_ptr), ("bn_wq", c_ptr), ("bn_bq", c_ptr),
                ("bn_neg_min", c_float), ("bn_min", c_float), ("bn_scale", c_float), ("bn_qmax", c_float),
                ("residual", c_ptr), ("relu", c_int), ("out_f32", c_ptr), ("out_bncode", c_ptr),
                ("out_code0", c_ptr), ("code0_cp", c_int), ("code0_pad", c_int), ("code0_hp", c_int),
                ("code0_wp", c_int), ("code0_neg_min", c_float), ("code0_scale", c_float), ("code0_qmax", c_float),
                ("out_code1", c_ptr), ("code1_cp", c_int), ("code1_pad", c_int), ("code1_hp", c_int),
                ("code1_wp", c_int), ("code1_neg_min", c_float), ("code1_scale", c_float), ("code1_qmax", c_float),
                ("lut", c_ptr), ("f32_tiled", c_int), ("nres", c_int), ("res_relu0", c_int),
                ("res", ResLink * MAX_RES), ("bncode_tiled", c_int)]

class BnParams(ctypes.Structure):
    """qnn_bn_params (include/qnn.h)."""
    _fields_ = [("mean", c_ptr), ("sq", c_ptr), ("wq", c_ptr), ("bq", c_ptr), ("neg_min", c_float),
                ("min", c_float), ("scale", c_float), ("qmax", c_float)]


class CodeOut(ctypes.Structure):
    """qnn_code_out (include/qnn.h)."""
    _fields_ = [("ptr", c_ptr), ("cp", c_int), ("pad", c_int), ("hp", c_int), ("wp", c_int), ("neg_min", c_float),
                ("scale", c_float), ("qmax", c_float)]


_PB, _PC = ctypes.POINTER(BnParams), ctypes.POINTER(CodeOut)

# name -> argtypes (restype is int status for all but the two metadata calls)
SIGNATURES = {
    "qnn_fake_quant_f32": [c_ptr, c_ptr, c_i64, c_float, c_float, c_float, c_float, c_ptr],
    "qnn_fake_quant_rows_f32": [c_ptr, c_ptr, c_int, c_i64, c_ptr, c_ptr, c_float, c_ptr],
    "qnn_fake_quant_vec_f32": [c_ptr, c_ptr, c_int, c_float, c_int, c_ptr, c_ptr],
    "qnn_grad_quant_f32": [c_ptr, c_ptr, c_ptr, ctypes.c_int64, c_float, c_float, c_float, c_ptr],
    "qnn_quantize_nchw_to_nhwc8": [c_ptr, c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                   c_float, c_ptr],
    "qnn_quantize_nchw_to_s2d8": [c_ptr, c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                  c_float, c_ptr],
    "qnn_pack_weight_i8": [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_ptr, c_ptr, c_ptr,
                           c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    "qnn_conv_border_table": [c_ptr, c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_int, c_float, c_ptr, c_ptr],
    "qnn_qconv2d_fwd": [c_ptr, c_ptr, ctypes.POINTER(ConvDesc), ctypes.POINTER(Epilogue), c_ptr],
    "qnn_qconv2d_fwd_nchw_f32": [c_ptr, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_ptr,
                                 ctypes.POINTER(ConvDesc), ctypes.POINTER(Epilogue), c_int, c_ptr],
    "qnn_conv_plan": [ctypes.POINTER(ConvDesc), ctypes.POINTER(Epilogue), c_ptr, c_ptr, c_ptr, c_ptr],
    "qnn_conv_occupancy": [ctypes.POINTER(ConvDesc), ctypes.POINTER(Epilogue), c_ptr, c_ptr, c_ptr, c_ptr],
    "qnn_dwconv2d_fwd": [c_ptr, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_float, c_float, c_float, c_float, c_ptr, c_ptr, c_ptr],
    "qnn_qconv2d_maxpool_fwd": [c_ptr, c_ptr, ctypes.POINTER(ConvDesc), ctypes.POINTER(Epilogue), c_int, c_int, c_ptr,
                                c_ptr, _PC, c_ptr, _PC, c_ptr],
    "qnn_maxpool_bn": [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _PB, c_int, c_ptr,
                       c_int, c_ptr, c_ptr, _PC, c_ptr, _PC, c_ptr],
    "qnn_dwconv_fused": [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_float, c_float, c_ptr, _PB, c_int, c_ptr, _PC, c_ptr],
    "qnn_dwconv_fused_generic": [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_float, c_float, c_ptr, _PB, c_int, c_ptr, _PC, c_ptr],
    "qnn_dwconv_fused_lut": [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int,
                             c_int, c_int, c_int, c_int, c_float, c_float, c_ptr, _PB, c_ptr, _PC, c_ptr],
    "qnn_avgpool_quant": [c_ptr, c_int, c_int, c_int, c_int, c_ptr, _PC, c_ptr],
    "qnn_bn_code_lut": [_PB, c_int, c_int, _PC, c_ptr, c_ptr],
    "qnn_chain_epilogue": [c_ptr, c_int, c_int, c_int, c_int, ctypes.POINTER(Epilogue), c_ptr],
    "qnn_qconv2d_generic_fwd": [c_ptr, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_ptr, c_int,
                                c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr,
                                c_ptr, c_ptr],
    "qnn_comm_unique_id": [c_ptr, ctypes.c_size_t],
    "qnn_comm_init": [c_int, c_int, c_ptr],
    "qnn_gather_f32": [c_ptr, c_ptr, ctypes.c_size_t, c_int, c_ptr],
    "qnn_comm_destroy": [],
    "qnn_measure_stats_f32": [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr],
    "qnn_rangebn_stats_f32": [c_ptr, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    "qnn_device_errors": [c_ptr, c_int],
    "qnn_debug_set_spin_limit": [c_int],
    "qnn_rangebn_f32": [c_ptr, c_ptr, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_ptr, c_ptr, c_ptr,
                        c_ptr, c_ptr, c_int, c_ptr],
}


class QnnLibraryError(RuntimeError):
    pass


DEVERR_PB_SPIN = 1  # QNN_DEVERR_PB_SPIN


def device_errors(clear=True):
    """The device error word (include/qnn.h qnn_device_errors; synchronizes the device)."""
    v = ctypes.c_uint32(0)
    call("qnn_device_errors", ctypes.byref(v), 1 if clear else 0)
    return v.value


class QnnError(RuntimeError):
    pass


_lib = None


def load(path=None):
    """Load and type the library (cached).  Raises QnnLibraryError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise QnnLibraryError(
            f"qnn: {path} not found - build it with `make -C quantized.pytorch_amd` "
            "(the int8 MI355X path has no fallback)")
    lib = ctypes.CDLL(path)
    lib.qnn_abi_version.restype = c_int
    lib.qnn_abi_version.argtypes = []
    lib.qnn_last_error.restype = ctypes.c_char_p
    lib.qnn_last_error.argtypes = []
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = c_int
    v = lib.qnn_abi_version()
    if v != ABI_VERSION:
        raise QnnLibraryError(f"qnn: ABI version mismatch (library {v}, bindings {ABI_VERSION})")
    lib.qnn_measure_stats_work.restype = c_i64
    lib.qnn_measure_stats_work.argtypes = [c_i64]
    lib.qnn_conv_tile_count.restype = c_int
    lib.qnn_conv_tile_count.argtypes = []
    lib.qnn_conv_tile_kernel.restype = ctypes.c_char_p
    lib.qnn_conv_tile_kernel.argtypes = [c_int]
    if lib.qnn_conv_tile_count() != CONV_TILES:
        raise QnnLibraryError(f"qnn: library has {lib.qnn_conv_tile_count()} conv tile configurations, "
                              f"bindings expect {CONV_TILES}")
    _lib = lib
    return lib


def tile_kernel(cfg):
    """Kernel family (device function name) of tile configuration `cfg` (0-based, as
    qnn_conv_plan reports it): qnn_conv_tile_kernel."""
    n = load().qnn_conv_tile_kernel(int(cfg))
    if n is None:
        raise QnnError(f"qnn: no tile configuration {cfg}")
    return n.decode()


def tile_ids(kernel):
    """The 0-based tile configurations of one kernel family, in id order."""
    return [k for k in range(CONV_TILES) if tile_kernel(k) == kernel]


class LaunchTimer:
    """Optional per-launch HIP-event timing of selected entry points (bench/profiling).

    Events are recorded on the current PyTorch stream, which is the stream every
    qnn call is issued on, so they bracket exactly that launch.
    """

    def __init__(self, names):
        self.names = set(names)
        self.records = []

    def durations_ms(self):
        torch.cuda.synchronize()
        return [(n, a.elapsed_time(b)) for n, a, b in self.records]


_timer = None


def set_timer(timer):
    global _timer
    _timer = timer


def call(name, *args):
    """Invoke a C-ABI entry point and raise QnnError on a non-zero status."""
    lib = load()
    t = _timer
    if t is not None and name in t.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib, name)(*args)
        e1.record()
        t.records.append((name, e0, e1))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.qnn_last_error().decode(errors="replace")
        raise QnnError(f"{name} failed (status {rc}): {msg}")


STATUS_UNSUPPORTED = 3  # QNN_ERR_UNSUPPORTED (include/qnn.h)


def call_unsupported_ok(name, *args):
    """call(), except that QNN_ERR_UNSUPPORTED is returned (False) instead of raised: for entry
    points the caller has a fallback for.  True when the call ran."""
    lib = load()
    t = _timer
    if t is not None and name in t.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib, name)(*args)
        e1.record()
        if rc == 0:
            t.records.append((name, e0, e1))
    else:
        rc = getattr(lib, name)(*args)
    if rc == STATUS_UNSUPPORTED:
        return False
    if rc != 0:
        msg = lib.qnn_last_error().decode(errors="replace")
        raise QnnError(f"{name} failed (status {rc}): {msg}")
    return True


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t):
    """hipStream_t of the current PyTorch stream on t's device."""
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
