"""Run-time loader for the read-only reference (test-fixture generation only).

The reference (`/root/reference`) imports two things that are absent offline:

* the un-vendored `utils` git submodule (`.gitmodules:1-4`), of which
  `models/modules/quantize.py:7-12` only needs import-time names;
* `torchvision.transforms` (`models/resnet_quantized.py:2`,
  `models/mobilenet_quantized.py:7,122-137`), used only to build the
  `input_transform` dict.

None of those names is on the eval hot path.  This module
registers in-memory stand-ins for them, registers a bare `models` package whose
`__path__` points at the reference so that `models/__init__.py` (which imports
every model zoo file) never runs, and imports the three hot-path files.  It
contains no reference code and does nothing when `/root/reference` is absent.

Used only by `tools/gen_golden.py`; never by the product, tests, bench or smoke.
"""
import functools
import importlib
import os
import sys
import types

REF = os.environ.get("QNN_REFERENCE", "/root/reference")


def _stub_utils():
    utils = types.ModuleType("utils")
    utils.__path__ = []

    absorb = types.ModuleType("utils.absorb_bn")

    def _nyi(*a, **k):
        raise NotImplementedError("utils submodule is not vendored")

    absorb.absorb_bn = _nyi
    absorb.absorb_bn_step = _nyi

    misc = types.ModuleType("utils.misc")
    misc.get_lambda_module_class = _nyi

    pc = types.ModuleType("utils.partial_class")

    def partial_class(cls, *args, **kwargs):
        class _P(cls):
            __init__ = functools.partialmethod(cls.__init__, *args, **kwargs)
        return _P

    pc.partial_class = partial_class

    mr = types.ModuleType("utils.module_rewriter")

    class ReWriter:
        def __init__(self, verbose=0):
            self._default_cfgs = {}
            self.group_fns = {}

        def gen_builder_fn(self, c):
            return c

    class _Matcher:
        def __init__(self, *a, **k):
            pass

    class BaseConfigurationGroup:
        def __init__(self, name, matcher, builder_fn=None):
            self.name, self.matcher, self.builder_fn = name, matcher, builder_fn

    mr.ReWriter = ReWriter
    mr.BaseMatcher = mr.FirstNMatcher = mr.ExactAttrMatcher = mr.BasicTypeMatcher = _Matcher
    mr.BaseConfigurationGroup = BaseConfigurationGroup

    for m in (utils, absorb, misc, pc, mr):
        sys.modules[m.__name__] = m


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tv.__path__ = []
    tr = types.ModuleType("torchvision.transforms")

    class _T:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    for n in ("Normalize", "Compose", "RandomResizedCrop", "RandomHorizontalFlip",
              "ToTensor", "Resize", "CenterCrop", "RandomCrop", "Scale"):
        setattr(tr, n, _T)
    tv.transforms = tr
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tr


def load():
    """Return (quantize, resnet_quantized, mobilenet_quantized) reference modules."""
    if not os.path.isdir(os.path.join(REF, "models")):
        raise FileNotFoundError(f"reference not found at {REF}")
    sys.dont_write_bytecode = True
    if "utils.module_rewriter" not in sys.modules:
        _stub_utils()
    if "torchvision.transforms" not in sys.modules:
        _stub_torchvision()
    if "models" not in sys.modules:
        pkg = types.ModuleType("models")
        pkg.__path__ = [os.path.join(REF, "models")]
        sys.modules["models"] = pkg
    import warnings
    warnings.simplefilter("ignore")
    Q = importlib.import_module("models.modules.quantize")
    RQ = importlib.import_module("models.resnet_quantized")
    MQ = importlib.import_module("models.mobilenet_quantized")
    return Q, RQ, MQ
