"""qnn_avgpool_quant (resnet_quantized.py:153, mobilenet_quantized.py:157): the engine's global
average pool, from an NHWC map and from a C-tile map, bitwise torch's
AvgPool2d on the device, and the classifier's input codes bitwise the quantizer's."""
import pytest
import torch
import torch.nn.functional as F

from qnn import _lib
from qnn.engine import ctile_numel

pytestmark = pytest.mark.gpu


def _tile(xm, M, C):
    """[M][C] row-major -> the C-tile layout (inverse of qnn.engine.untile)."""
    mt, ct = -(-M // 32), -(-C // 32)
    buf = torch.zeros(ctile_numel(M, C), dtype=torch.float32, device=xm.device)
    full = torch.zeros(mt * 32, ct * 32, dtype=torch.float32, device=xm.device)
    full[:M, :C] = xm
    # [mt][32 m][ct][4 g][2 h][4 u] -> [mt][ct][g][h][m][u]
    t = full.view(mt, 32, ct, 4, 2, 4).permute(0, 2, 3, 4, 1, 5).reshape(-1)
    buf[:t.numel()] = t
    return buf


@pytest.mark.parametrize("n,hw,c", [(5, 49, 512), (3, 49, 1024), (4, 64, 64), (2, 9, 96), (3, 49, 2048)])
def test_avgpool_tiled_bitwise(gpu, n, hw, c):
    g = torch.Generator().manual_seed(n * 1000 + hw + c)
    k = int(hw ** 0.5)
    x = (torch.randn(n, c, k, k, generator=g) * 3).to(gpu)
    ref = F.avg_pool2d(x, k).reshape(n, c)
    xm = x.permute(0, 2, 3, 1).reshape(n * hw, c).contiguous()
    st = _lib.stream_of(x)
    outs = {}
    for tiled in (0, 1):
        src = _tile(xm, n * hw, c) if tiled else xm
        y = torch.full((n, c), float("nan"), dtype=torch.float32, device=gpu)
        codes = torch.full((n * c + 128,), 77, dtype=torch.int8, device=gpu)
        co = _lib.CodeOut(ptr=codes.data_ptr(), cp=c, pad=0, hp=1, wp=1, neg_min=2.0, scale=4.0 / 255, qmax=255.0)
        _lib.call("qnn_avgpool_quant", _lib.ptr(src), n, hw, c, tiled, _lib.ptr(y), co, st)
        torch.cuda.synchronize()
        outs[tiled] = (y, codes[: n * c].clone())
    assert torch.equal(outs[0][0], ref) and torch.equal(outs[1][0], ref)
    assert torch.equal(outs[0][1], outs[1][1])
