"""ResNet builders with the module tree of models/resnet_quantized.py.

Identical attribute names, registration order and therefore state_dict keys
(reference checkpoints load with strict=True), built from this package's
QConv2d / QLinear / RangeBN.  Bit widths and biprecision are the reference's
module constants (resnet_quantized.py:7-10).  The block forwards are the
reference graphs (:52-68, :93-113, :140-155); for a fused single-pass inference
of the whole network see `qnn.engine`.
"""
import math

import torch.nn as nn

from .dispatch import engine_forward
from .quantize import QConv2d, QLinear, RangeBN, quantize, quantize_grad  # noqa: F401

__all__ = ["resnet_quantized"]

NUM_BITS = 8
NUM_BITS_WEIGHT = 8
NUM_BITS_GRAD = 8
BIPRECISION = True

_Q = dict(num_bits=NUM_BITS, num_bits_weight=NUM_BITS_WEIGHT, num_bits_grad=NUM_BITS_GRAD, biprecision=BIPRECISION)


def _rbn(c):
    return RangeBN(c, num_bits=NUM_BITS, num_bits_grad=NUM_BITS_GRAD)


def conv3x3(in_planes, out_planes, stride=1):
    "3x3 convolution with padding (resnet_quantized.py:13-16)"
    return QConv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False, **_Q)


def init_model(model):
    """resnet_quantized.py:19-34 (torch RNG); see qnn.synthetic for the
    deterministic synthetic initialisation used by tests and the benchmark."""
    for m in model.modules():
        if isinstance(m, QConv2d):
            fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
            m.weight.data.normal_(0, math.sqrt(2.0 / fan))
        elif isinstance(m, RangeBN):
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    for m in model.modules():
        if isinstance(m, Bottleneck):
            nn.init.constant_(m.bn3.weight, 0)
        elif isinstance(m, BasicBlock):
            nn.init.constant_(m.bn2.weight, 0)
    model.fc.weight.data.normal_(0, 0.01)
    model.fc.bias.data.zero_()


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = _rbn(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _rbn(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        shortcut = x if self.downsample is None else self.downsample(x)
        out += shortcut
        return self.relu(out)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = QConv2d(inplanes, planes, kernel_size=1, bias=False, **_Q)
        self.bn1 = _rbn(planes)
        self.conv2 = QConv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False, **_Q)
        self.bn2 = _rbn(planes)
        self.conv3 = QConv2d(planes, planes * 4, kernel_size=1, bias=False, **_Q)
        self.bn3 = _rbn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        shortcut = x if self.downsample is None else self.downsample(x)
        out += shortcut
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self):
        super().__init__()

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                QConv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False, **_Q),
                _rbn(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        y = engine_forward(self, x)  # a plain eval forward on the cached fused engine (qnn/dispatch.py)
        if y is not None:
            return y
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = self.avgpool(x)
        return self.fc(x.view(x.size(0), -1))

    @staticmethod
    def regularization(model, weight_decay=1e-4):
        l2_params = 0
        for m in model.modules():
            if isinstance(m, nn.Conv2d) or isinstance(m, nn.Linear):
                l2_params += m.weight.pow(2).sum()
                if m.bias is not None:
                    l2_params += m.bias.pow(2).sum()
        return weight_decay * 0.5 * l2_params


class ResNet_imagenet(ResNet):
    def __init__(self, num_classes=1000, block=Bottleneck, layers=(3, 4, 23, 3)):
        super().__init__()
        self.inplanes = 64
        self.conv1 = QConv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False, **_Q)
        self.bn1 = _rbn(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AvgPool2d(7)
        self.fc = QLinear(512 * block.expansion, num_classes, **_Q)
        init_model(self)
        scale = 256.0 / 256.0

        def ramp_up_lr(lr0, lrT, T):
            rate = (lrT - lr0) / T
            return "lambda t: {'lr': %s + t * %s}" % (lr0, rate)

        self.regime = [
            {"epoch": 0, "optimizer": "SGD", "momentum": 0.9, "step_lambda": ramp_up_lr(0, 0.1 * scale, 5004 * 5 / scale)},
            {"epoch": 5, "lr": scale * 1e-1},
            {"epoch": 30, "lr": scale * 1e-2},
            {"epoch": 60, "lr": scale * 1e-3},
            {"epoch": 80, "lr": scale * 1e-4},
        ]


class ResNet_cifar10(ResNet):
    def __init__(self, num_classes=10, block=BasicBlock, depth=18):
        super().__init__()
        self.inplanes = 16
        n = int((depth - 2) / 6)
        self.conv1 = QConv2d(3, 16, kernel_size=3, stride=1, padding=1, bias=False, **_Q)
        self.bn1 = _rbn(16)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = lambda x: x
        self.layer1 = self._make_layer(block, 16, n)
        self.layer2 = self._make_layer(block, 32, n, stride=2)
        self.layer3 = self._make_layer(block, 64, n, stride=2)
        self.layer4 = lambda x: x
        self.avgpool = nn.AvgPool2d(8)
        self.fc = QLinear(64, num_classes, **_Q)
        init_model(self)
        self.regime = [
            {"epoch": 0, "optimizer": "SGD", "lr": 1e-1, "weight_decay": 1e-4, "momentum": 0.9},
            {"epoch": 81, "lr": 1e-2},
            {"epoch": 122, "lr": 1e-3, "weight_decay": 0},
            {"epoch": 164, "lr": 1e-4},
        ]


_IMAGENET = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]), 50: (Bottleneck, [3, 4, 6, 3]),
             101: (Bottleneck, [3, 4, 23, 3]), 152: (Bottleneck, [3, 8, 36, 3])}


def resnet_quantized(**kwargs):
    """resnet_quantized.py:235-261: dataset 'imagenet' (depth 18/34/50/101/152,
    default 50) or 'cifar10' (default depth 56); returns None otherwise."""
    num_classes, depth, dataset = map(kwargs.get, ["num_classes", "depth", "dataset"])
    if dataset == "imagenet":
        num_classes = num_classes or 1000
        depth = depth or 50
        if depth in _IMAGENET:
            block, layers = _IMAGENET[depth]
            return ResNet_imagenet(num_classes=num_classes, block=block, layers=layers)
        return None
    if dataset == "cifar10":
        num_classes = num_classes or 10
        depth = depth or 56
        return ResNet_cifar10(num_classes=num_classes, block=BasicBlock, depth=depth)
    return None
