"""The drop-in QConv2d for the shapes the int8 MFMA path does not take (missing #3):
dilation != 1, grouped convs other than depthwise, unequal and string padding, padding_mode --
the reference's forward is F.conv2d(input_, qweight, qbias, stride, padding, dilation, groups)
(quantize.py:342-344), which never applies padding_mode.  Checked against the oracle's restatement
of that forward (oracle.qnn_oracle.qconv2d) with the per-layer bar of every other conv test.
"""
import pytest
import torch

from oracle import qnn_oracle as O
from qnn import synthetic
from qnn.quantize import QConv2d

pytestmark = pytest.mark.gpu
LAYER_TOL = 1e-5
XR = (-1.25, 2.0)


def _layer(cin, cout, k, **kw):
    m = QConv2d(cin, cout, k, **kw)
    synthetic.init_params(m, 21)
    m.quantize_input.running_min.fill_(XR[0])
    m.quantize_input.running_max.fill_(XR[1])
    return m.eval()


@pytest.mark.parametrize("cin,cout,k,kw", [
    (8, 16, 3, dict(padding=2, dilation=2)),                 # dilated (DeepLab-style)
    (8, 8, 3, dict(padding=(1, 2), dilation=(1, 2), stride=2)),
    (8, 16, 3, dict(padding=1, groups=4)),                   # grouped, 2 channels per group
    (12, 6, (3, 5), dict(padding=(1, 2), groups=3, bias=False)),
    (6, 8, (3, 1), dict(padding=(1, 0))),                    # unequal padding
    (8, 8, 4, dict(padding="same")),                          # 'same', even kernel: odd extra bottom/right
    (8, 8, 3, dict(padding="valid", stride=(2, 1))),
    (8, 8, 3, dict(padding=1, padding_mode="reflect")),       # the reference pads with zeros anyway
])
def test_generic_conv_matches_reference(gpu, cin, cout, k, kw):
    m = _layer(cin, cout, k, **kw).to(gpu)
    x = synthetic.input_batch((3, cin, 11, 10), 22).to(gpu)
    with torch.no_grad():
        y = m(x)
    sd = {n: v.detach().cpu() for n, v in m.state_dict().items()}
    ref = O.qconv2d(x.cpu(), sd["weight"], sd.get("bias"), m.stride, m.padding, m.dilation, m.groups, XR)
    assert y.shape == ref.shape
    err = (y.cpu() - ref).abs().max().item()
    assert err <= LAYER_TOL * ref.abs().max().item() + 1e-6, err
    # the weight ranges the forward refreshed are the reference's per-channel ones (quantize.py:317-323)
    wmin, wmax = O.weight_ranges(sd["weight"])
    assert torch.equal(m.weight_min.cpu(), wmin) and torch.equal(m.weight_max.cpu(), wmax)
