"""ResNet-50 (v1.5: stride on the 3x3 conv), the reference's headline ImageNet workload
(examples/imagenet/main_amp.py, ``-a resnet50``). Written here because torchvision is not part of
the stack; layer shapes and init follow torchvision's ``resnet50`` so parameter counts (25.56 M)
and FLOPs match.
"""
from __future__ import annotations

from typing import List, Optional, Type

import torch
import torch.nn as nn


def conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample: Optional[nn.Module] = None,
                 norm_layer=nn.BatchNorm2d, fused=False):
        super().__init__()
        self.fused = fused
        relu_kw = {"fuse_relu": True} if fused else {}
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = norm_layer(planes, **relu_kw)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = norm_layer(planes, **relu_kw)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion, **relu_kw)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        if self.fused:
            # BN+ReLU and BN+residual-add+ReLU run as single fused passes (SyncBatchNorm fuse_relu)
            out = self.bn1(self.conv1(x))
            out = self.bn2(self.conv2(out))
            if self.downsample is not None:
                identity = self.downsample(x)
            return self.bn3(self.conv3(out), z=identity)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = out + identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block: Type[Bottleneck], layers: List[int], num_classes=1000,
                 zero_init_residual=False, norm_layer=nn.BatchNorm2d, fused=False):
        super().__init__()
        self._norm_layer = norm_layer
        self.fused = fused
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(64, fuse_relu=True) if fused else norm_layer(64)
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
            elif isinstance(m, nn.modules.batchnorm._BatchNorm):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, norm_layer, fused=self.fused)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, norm_layer=norm_layer, fused=self.fused))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.bn1(self.conv1(x)) if self.fused else self.relu(self.bn1(self.conv1(x)))
        x = self.maxpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet50(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet50_fused(process_group=None, channel_last=True, **kw) -> ResNet:
    """ResNet-50 whose BatchNorms are fused SyncBatchNorms (BN+ReLU and BN+add+ReLU in one pass),
    synchronised over ``process_group`` -- the 'amp O2 + SyncBatchNorm' benchmark model."""
    from ..parallel import SyncBatchNorm

    def norm(c, fuse_relu=False):
        return SyncBatchNorm(c, process_group=process_group, channel_last=channel_last, fuse_relu=fuse_relu)

    return ResNet(Bottleneck, [3, 4, 6, 3], norm_layer=norm, fused=True, **kw)


def resnet18_like(**kw) -> ResNet:
    """Small bottleneck ResNet used by fast tests (same block structure, fewer blocks)."""
    return ResNet(Bottleneck, [1, 1, 1, 1], **kw)
