"""ResNet-18 / ResNet-50 (torchvision architecture and state_dict names) on ringdp's NHWC kernels.

Reference: ``torchvision.models.resnet18(pretrained=False, num_classes=10)`` in
``ref/example_mp.py:50`` and ``ref/example_launch.py:26`` (the ImageNet stem
7x7/s2 + maxpool applied to 32x32 CIFAR inputs, so layer4 runs at 1x1); ResNet-50 for BASELINE
config 4.  torchvision is not part of this stack, so the architecture is defined here with the
same module tree (``conv1 bn1 layer1..4 fc``, blocks ``conv1 bn1 conv2 bn2 [conv3 bn3] downsample``)
and the same initialisation (kaiming-normal fan_out convs, BN weight 1 / bias 0).

GPU: activations are NHWC bf16 and every conv+BN(+residual)(+ReLU) is one fused implicit-GEMM
forward + one elementwise launch (``ringdp.ops.nhwc``); CPU: the plain ATen forward (reference
semantics, test oracle).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.nhwc import (ConvBNAct, ConvBNActFork, ConvBNActPair, MaxPoolNHWC, classifier_head, pack_conv_weights,
                        to_nhwc)

# {id(conv): (krsc, crsk)} of the forward in progress (ResNet.forward_nhwc packs every conv weight in one
# launch); empty outside it, so blocks called on their own pack per conv
_PACKED: dict = {}


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _bn_args(bn: nn.BatchNorm2d):
    """(momentum, num_batches_tracked to increment on device or None, running_mean, running_var)."""
    count = bn.training and bn.track_running_stats and bn.num_batches_tracked is not None
    nbt = None
    if bn.momentum is not None:
        momentum = bn.momentum
        nbt = bn.num_batches_tracked if count else None  # incremented by the BN kernel (no extra launch)
    elif count:
        # cumulative moving average (torch's exponential_average_factor for momentum=None);
        # reads the incremented counter on the host, as upstream does
        bn.num_batches_tracked.add_(1)
        momentum = 1.0 / float(bn.num_batches_tracked.item())
    else:
        momentum = 0.0
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return momentum, nbt, rm, rv


def _fused(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool, residual=None):
    momentum, nbt, rm, rv = _bn_args(bn)
    return ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, residual, rm, rv, conv.stride[0], conv.padding[0],
                           relu, bn.training, momentum, bn.eps, nbt, _PACKED.get(id(conv)))


def _fused_fork(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool):
    """(conv+BN(+ReLU) of x, x as the identity shortcut) - the shortcut's gradient joins the conv's data
    gradient in its GEMM epilogue."""
    momentum, nbt, rm, rv = _bn_args(bn)
    return ConvBNActFork.apply(x, conv.weight, bn.weight, bn.bias, rm, rv, conv.stride[0], conv.padding[0], relu,
                               bn.training, momentum, bn.eps, nbt, _PACKED.get(id(conv)))


def _fused_pair(x, conv1: nn.Conv2d, bn1: nn.BatchNorm2d, relu1: bool, conv2: nn.Conv2d, bn2: nn.BatchNorm2d,
                relu2: bool):
    """Two conv+BN branches of one input (first conv + projection shortcut)."""
    m1, n1, rm1, rv1 = _bn_args(bn1)
    m2, n2, rm2, rv2 = _bn_args(bn2)
    return ConvBNActPair.apply(x, conv1.weight, bn1.weight, bn1.bias, rm1, rv1, n1, conv2.weight, bn2.weight, bn2.bias,
                               rm2, rv2, n2, (conv1.stride[0], conv1.padding[0], relu1, m1),
                               (conv2.stride[0], conv2.padding[0], relu2, m2), bn1.training, bn1.eps, bn2.eps,
                               _PACKED.get(id(conv1)), _PACKED.get(id(conv2)))


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):  # ATen (CPU) path
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)

    def forward_nhwc(self, x):
        if self.downsample is None:
            out, identity = _fused_fork(x, self.conv1, self.bn1, True)
        else:
            out, identity = _fused_pair(x, self.conv1, self.bn1, True, self.downsample[0], self.downsample[1], False)
        return _fused(out, self.conv2, self.bn2, True, identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)

    def forward_nhwc(self, x):
        if self.downsample is None:
            out, identity = _fused_fork(x, self.conv1, self.bn1, True)
        else:
            out, identity = _fused_pair(x, self.conv1, self.bn1, True, self.downsample[0], self.downsample[1], False)
        out = _fused(out, self.conv2, self.bn2, True)
        return _fused(out, self.conv3, self.bn3, True, identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return self.forward_nhwc(x)
        return self.reference_forward(x)

    def reference_forward(self, x: torch.Tensor) -> torch.Tensor:
        """ATen NCHW forward (CPU path and numerics oracle)."""
        x = self.maxpool(self.relu(self.bn1(self.conv1(x.to(self.conv1.weight.dtype)))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """``x``: NCHW images (fp32/bf16), converted to NHWC bf16 + channel-padded on device."""
        h = to_nhwc(x)
        _PACKED.update(pack_conv_weights(m for m in self.modules() if isinstance(m, nn.Conv2d)))
        try:
            h = _fused(h, self.conv1, self.bn1, True)
            h = MaxPoolNHWC.apply(h, 3, 2, 1)
            for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
                for blk in layer:
                    h = blk.forward_nhwc(h)
        finally:
            _PACKED.clear()
        return classifier_head(h, self.fc)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)
