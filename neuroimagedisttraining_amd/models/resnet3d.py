"""3D ResNets for volumetric MRI.

* :class:`ResNet_l3` — the reference's 3-stage 3D ResNet (``fedml_api/model/cv/salient_models.py:8-139``,
  conv k3 s2 p3 stem, max-pool, 64/128/256 stages, ``AvgPool3d(3)``, fc -> 512 -> C, returns ``[x, x1]``).
  The reference hard-codes ``fc`` to ``9216*expansion`` inputs, which does not match a 121x145x121 volume
  (3072*expansion features, quirk Q18); here the flattened size is computed from ``in_shape`` so the model
  actually runs on ABCD-shape data (``fc_in=9216*expansion`` restores the reference constant).
* :func:`resnet3d_50` — a standard 4-stage bottleneck 3D ResNet-50 for BASELINE.json config 5 (new), with
  optional activation checkpointing per stage for full-resolution volumes.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv3d(in_planes, out_planes, 3, stride, 1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm3d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm3d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv3d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm3d(planes)
        self.conv2 = nn.Conv3d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm3d(planes)
        self.conv3 = nn.Conv3d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm3d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


def _make_layer(owner, block, planes, blocks, stride=1):
    down = None
    if stride != 1 or owner.inplanes != planes * block.expansion:
        down = nn.Sequential(nn.Conv3d(owner.inplanes, planes * block.expansion, 1, stride, bias=False),
                             nn.BatchNorm3d(planes * block.expansion))
    layers = [block(owner.inplanes, planes, stride, down)]
    owner.inplanes = planes * block.expansion
    layers += [block(owner.inplanes, planes) for _ in range(1, blocks)]
    return nn.Sequential(*layers)


def _init(model):
    for m in model.modules():
        if isinstance(m, nn.Conv3d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm3d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)


class ResNet_l3(nn.Module):
    def __init__(self, block, layers, num_classes, in_shape=(121, 145, 121), fc_in=None):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv3d(1, 64, 3, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm3d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool3d(3, 2, 1)
        self.layer1 = _make_layer(self, block, 64, layers[0])
        self.layer2 = _make_layer(self, block, 128, layers[1], 2)
        self.layer3 = _make_layer(self, block, 256, layers[2], 2)
        self.avgpool = nn.AvgPool3d(3)
        if fc_in is None:
            fc_in = self._flat(in_shape)
        self.fc = nn.Linear(fc_in, 512)
        self.fc2 = nn.Linear(512, num_classes)
        _init(self)

    def _flat(self, shape):
        def o(n, k, s, p):
            return (n + 2 * p - k) // s + 1
        dims = []
        for n in shape:
            n = o(n, 3, 2, 3)     # conv1
            n = o(n, 3, 2, 1)     # maxpool
            n = o(n, 3, 2, 1)     # layer2 stride
            n = o(n, 3, 2, 1)     # layer3 stride
            n = n // 3            # avgpool(3)
            dims.append(n)
        return 256 * self.layer3[0].expansion * dims[0] * dims[1] * dims[2]

    def features(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer3(self.layer2(self.layer1(x)))
        return self.avgpool(x).flatten(1)

    def forward(self, x):
        x1 = self.fc(self.features(x))
        return [self.fc2(x1), x1]


def resnet_l3(num_classes=1, block="basic", in_shape=(121, 145, 121)):
    b = BasicBlock if block == "basic" else Bottleneck
    return ResNet_l3(b, [2, 2, 2], num_classes, in_shape=in_shape)


class ResNet3D(nn.Module):
    """Four-stage 3D ResNet (ResNet-50 with Bottleneck [3,4,6,3]); ``checkpoint_stages`` trades recompute for
    activation memory at full 121x145x121 resolution."""

    def __init__(self, block, layers, num_classes=1, in_ch=1, width=64, checkpoint_stages=False):
        super().__init__()
        self.inplanes = width
        self.checkpoint_stages = checkpoint_stages
        self.conv1 = nn.Conv3d(in_ch, width, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm3d(width)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool3d(3, 2, 1)
        self.layer1 = _make_layer(self, block, width, layers[0])
        self.layer2 = _make_layer(self, block, width * 2, layers[1], 2)
        self.layer3 = _make_layer(self, block, width * 4, layers[2], 2)
        self.layer4 = _make_layer(self, block, width * 8, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool3d(1)
        self.fc = nn.Linear(width * 8 * block.expansion, num_classes)
        _init(self)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        for st in (self.layer1, self.layer2, self.layer3, self.layer4):
            if self.checkpoint_stages and self.training and x.requires_grad:
                x = checkpoint(st, x, use_reentrant=False)
            else:
                x = st(x)
        return self.fc(self.avgpool(x).flatten(1))


def resnet3d_50(num_classes=1, checkpoint_stages=False, width=64):
    return ResNet3D(Bottleneck, [3, 4, 6, 3], num_classes, width=width, checkpoint_stages=checkpoint_stages)


def resnet3d_18(num_classes=1, checkpoint_stages=False, width=64):
    return ResNet3D(BasicBlock, [2, 2, 2, 2], num_classes, width=width, checkpoint_stages=checkpoint_stages)
