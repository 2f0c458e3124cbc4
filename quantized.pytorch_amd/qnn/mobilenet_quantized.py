"""MobileNet-v1 builder with the module tree of models/mobilenet_quantized.py.

Same attributes and state_dict keys (`features.<i>[.components.<j>]`,
`avg_pool`, `fc`).  The depthwise QConv2d keeps bias=True, so its bias is
fake-quantized (mobilenet_quantized.py:38-40); it runs on qnn's depthwise
kernel, the pointwise 1x1 convs on the int8 MFMA kernel.
"""
import math

import torch.nn as nn

from .dispatch import engine_forward
from .quantize import QConv2d, QLinear, RangeBN, quantize, quantize_grad  # noqa: F401

__all__ = ["mobilenet_quantized"]

NUM_BITS = 8
NUM_BITS_WEIGHT = 8
NUM_BITS_GRAD = 8
BIPRECISION = True

_Q = dict(num_bits=NUM_BITS, num_bits_weight=NUM_BITS_WEIGHT, num_bits_grad=NUM_BITS_GRAD, biprecision=BIPRECISION)


def nearby_int(n):
    return int(round(n))


def init_model(model):
    """mobilenet_quantized.py:20-30 (torch RNG)."""
    for m in model.modules():
        if isinstance(m, QConv2d):
            fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
            m.weight.data.normal_(0, math.sqrt(2.0 / fan))
        elif isinstance(m, RangeBN):
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    model.fc.weight.data.normal_(0, 0.01)
    model.fc.bias.data.zero_()


def _rbn(c):
    return RangeBN(c, num_bits=NUM_BITS, num_bits_grad=NUM_BITS_GRAD)


class DepthwiseSeparableFusedConv2d(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0):
        super().__init__()
        self.components = nn.Sequential(
            QConv2d(in_channels, in_channels, kernel_size, stride=stride, padding=padding, groups=in_channels, **_Q),
            _rbn(in_channels),
            nn.ReLU(),
            QConv2d(in_channels, out_channels, 1, bias=False, **_Q),
            _rbn(out_channels),
            nn.ReLU(),
        )

    def forward(self, x):
        return self.components(x)


def _input_transform():
    try:
        import torchvision.transforms as transforms
    except ImportError:  # torchvision is not part of this image; the transforms are data-side only
        return None
    normalize = transforms.Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    return {
        "train": transforms.Compose([transforms.RandomResizedCrop(224, scale=(0.3, 1.0)),
                                     transforms.RandomHorizontalFlip(), transforms.ToTensor(), normalize]),
        "eval": transforms.Compose([transforms.Resize(256), transforms.CenterCrop(224), transforms.ToTensor(),
                                    normalize]),
    }


class MobileNet(nn.Module):
    def __init__(self, width=1.0, shallow=False, num_classes=1000):
        super().__init__()
        num_classes = num_classes or 1000
        width = width or 1.0
        r = lambda c: nearby_int(width * c)
        layers = [
            QConv2d(3, r(32), kernel_size=3, stride=2, padding=1, bias=False, **_Q),
            _rbn(r(32)),
            nn.ReLU(inplace=True),
        ]
        plan = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2)]
        if not shallow:
            plan += [(512, 512, 1)] * 5  # 5x 512->512 depthwise-separable blocks
        plan += [(512, 1024, 2), (1024, 1024, 1)]
        layers += [DepthwiseSeparableFusedConv2d(r(a), r(b), kernel_size=3, stride=s, padding=1) for a, b, s in plan]
        self.features = nn.Sequential(*layers)
        self.avg_pool = nn.AvgPool2d(7)
        self.fc = QLinear(r(1024), num_classes, **_Q)
        self.input_transform = _input_transform()
        self.regime = [
            {"epoch": 0, "optimizer": "SGD", "lr": 1e-1, "momentum": 0.9},
            {"epoch": 30, "lr": 1e-2},
            {"epoch": 60, "lr": 1e-3},
            {"epoch": 80, "lr": 1e-4},
        ]

    @staticmethod
    def regularization(model, weight_decay=4e-5):
        l2_params = 0
        for m in model.modules():
            if isinstance(m, QConv2d) or isinstance(m, nn.Linear):
                l2_params += m.weight.pow(2).sum()
                if m.bias is not None:
                    l2_params += m.bias.pow(2).sum()
        return weight_decay * 0.5 * l2_params

    def forward(self, x):
        y = engine_forward(self, x)  # a plain eval forward on the cached fused engine (qnn/dispatch.py)
        if y is not None:
            return y
        x = self.avg_pool(self.features(x))
        return self.fc(x.view(x.size(0), -1))


def mobilenet_quantized(**kwargs):
    """mobilenet_quantized.py:163-173."""
    num_classes, width, alpha, shallow = map(kwargs.get, ["num_classes", "width", "alpha", "shallow"])
    return MobileNet(width=width, shallow=shallow, num_classes=num_classes)
