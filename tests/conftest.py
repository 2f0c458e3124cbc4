import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "quantized.pytorch_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# The module path's per-shape autotune (qnn.quantize.MODULE_AUTOTUNE) would time every tile
# configuration for each of the many fresh layers the tests build; the tests force or use the
# cost model's configuration instead (every configuration is checked on its own), and
# tests/test_gpu_tiles.py::test_module_autotune_bitwise covers the autotune itself.
os.environ.setdefault("QNN_MODULE_AUTOTUNE", "0")
# The reference-forward dispatch to the fused engine (qnn/dispatch.py) is tested on its own
# (tests/test_gpu_dispatch.py); elsewhere model(x) is the per-module path the tests check.
os.environ.setdefault("QNN_ENGINE_DISPATCH", "off")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and the built libqnn_hip.so")


def load_fixture(name):
    """Golden fixture (data only; no pickle)."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["config"] = json.loads(str(d["config"])) if "config" in d else None
    return d


def fixture_buffers(d):
    import torch
    return {k[4:]: torch.from_numpy(v.copy()) for k, v in d.items() if k.startswith("buf/")}


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from qnn import _lib
    _lib.load()  # fail loudly when the HIP library is missing on a GPU box
    return torch.device("cuda:0")
