"""qnn — MI355X-native int8 inference path for the QConv2d / QLinear forward of
amishacorns/quantized.pytorch (models/modules/quantize.py).

Import-light: the HIP library (libqnn_hip.so, C ABI in include/qnn.h) is loaded
on first use by `qnn._lib.load()`.
"""
from . import synthetic  # noqa: F401

__all__ = ["quantize", "resnet_quantized", "mobilenet_quantized", "synthetic", "engine"]


def __getattr__(name):
    if name in ("quantize", "resnet_quantized", "mobilenet_quantized", "engine", "dist", "_lib"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
