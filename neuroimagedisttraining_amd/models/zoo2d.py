"""2D CNN families and tabular models used by the reference's CIFAR / Tiny-ImageNet / EMNIST baselines.

State-dict keys match the reference modules so per-parameter masks (DisPFL / SubAvg / SalientGrads) and saved
states interoperate (reference files: ``fedml_api/model/cv/resnet.py:9-214``, ``vgg.py:14-82``,
``lenet5.py:4-46``, ``cnn.py:6-166``, ``cnn_cifar10.py:12-50``, ``cnn_meta.py:17-177``).  The reference builds its
GroupNorm ResNets by patching BatchNorm attributes after construction; here the normalisation layer is chosen
by a factory at construction time (same keys, no dead BN parameters).

``LogisticRegression`` is new (BASELINE.json config 1: 2-client FedAvg LR plumbing on tabular data).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def _norm2d(kind, c):
    if kind == "gn":
        return nn.GroupNorm(num_groups=32, num_channels=c)
    if kind == "bn":
        return nn.BatchNorm2d(c)
    raise ValueError(kind)


class BasicBlock(nn.Module):
    """3x3-3x3 residual block with a 1x1 projection shortcut when shape changes (keys conv1/bn1/conv2/bn2/shortcut)."""
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, norm="bn"):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = _norm2d(norm, planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = _norm2d(norm, planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(nn.Conv2d(in_planes, planes * self.expansion, 1, stride, bias=False),
                                          _norm2d(norm, planes * self.expansion))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + self.shortcut(x))


class ResNet(nn.Module):
    """CIFAR-style ResNet (3x3 stem, 4 stages, ``avg_pool2d(4)`` head) — ``resnet.py:41-88``."""

    def __init__(self, block, num_blocks, class_num=10, norm="bn", adaptive_pool=False, in_ch=3):
        super().__init__()
        self.in_planes = 64
        self.conv1 = nn.Conv2d(in_ch, 64, 3, 1, 1, bias=False)
        self.bn1 = _norm2d(norm, 64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1, norm)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2, norm)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2, norm)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2, norm)
        self.adaptive = adaptive_pool
        if adaptive_pool:
            self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.linear = nn.Linear(512 * block.expansion, class_num)

    def _make_layer(self, block, planes, n, stride, norm):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(block(self.in_planes, planes, s, norm))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        y = self.avgpool(y) if self.adaptive else F.avg_pool2d(y, 4)
        return self.linear(torch.flatten(y, 1))


def customized_resnet18(pretrained=False, class_num=10, progress=True):
    """ResNet-18 with GroupNorm(32) everywhere (the reference's federated default, ``resnet.py:91-124``)."""
    m = ResNet(BasicBlock, [2, 2, 2, 2], class_num=class_num, norm="gn")
    assert len(dict(m.named_parameters())) == len(m.state_dict()), "GN model must have no BN buffers"
    return m


def original_resnet18(pretrained=False, class_num=10, progress=True):
    return ResNet(BasicBlock, [2, 2, 2, 2], class_num=class_num, norm="bn")


def tiny_resnet18(pretrained=False, class_num=200, progress=True):
    """Tiny-ImageNet variant: GroupNorm + adaptive average pooling (``resnet.py:134-214``)."""
    return ResNet(BasicBlock, [2, 2, 2, 2], class_num=class_num, norm="gn", adaptive_pool=True)


tiny_ResNet = ResNet


# ------------------------------------------------------------------------------------------------
_VGG_CFG = {"A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
            "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]}


def make_layers(cfg, group_norm=True):
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers.append(nn.Conv2d(c, v, 3, padding=1))
            layers += ([nn.GroupNorm(32, v)] if group_norm else []) + [nn.ReLU(inplace=True)]
            c = v
    layers.append(nn.AvgPool2d(1, 1))
    return nn.Sequential(*layers)


class VGG(nn.Module):
    """GroupNorm VGG with a ``Linear(512, C)`` head and kaiming init (``vgg.py:14-43``)."""

    def __init__(self, features, num_classes=10, init_weights=True):
        super().__init__()
        self.features = features
        self.classifier = nn.Sequential(nn.Linear(512, num_classes))
        if init_weights:
            for m in self.modules():
                if isinstance(m, nn.Conv2d):
                    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                    if m.bias is not None:
                        nn.init.zeros_(m.bias)
                elif isinstance(m, nn.GroupNorm):
                    nn.init.ones_(m.weight)
                    nn.init.zeros_(m.bias)
                elif isinstance(m, nn.Linear):
                    nn.init.normal_(m.weight, 0, 0.01)
                    nn.init.zeros_(m.bias)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


def vgg11(num_class=10):
    return VGG(make_layers(_VGG_CFG["A"]), num_classes=num_class)


def vgg16(num_class=10):
    return VGG(make_layers(_VGG_CFG["D"]), num_classes=num_class)


# ------------------------------------------------------------------------------------------------
class LeNet5(nn.Module):
    """Caffe-style LeNet-5 for 1x28x28 inputs (``lenet5.py:4-26``)."""

    def __init__(self, class_num=10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5)
        self.conv2 = nn.Conv2d(20, 50, 5)
        self.fc3 = nn.Linear(50 * 4 * 4, 500)
        self.fc4 = nn.Linear(500, class_num)

    def forward(self, x):
        x = F.max_pool2d(self.conv1(x), 2)
        x = F.max_pool2d(self.conv2(x), 2)
        return self.fc4(F.relu(self.fc3(x.flatten(1))))


class LeNet5_cifar(nn.Module):
    """Classic LeNet for 3x32x32 (``lenet5.py:29-46``)."""

    def __init__(self, out_size=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 6, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, out_size)

    def forward(self, x):
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = F.relu(self.fc1(x.flatten(1)))
        return self.fc3(F.relu(self.fc2(x)))


class cnn_cifar10(nn.Module):
    """2x conv5 + 3 FC (``cnn_cifar10.py:12-30``)."""
    n_cls = 10

    def __init__(self, n_cls=None):
        super().__init__()
        if n_cls is not None:
            self.n_cls = n_cls
        self.conv1 = nn.Conv2d(3, 64, 5)
        self.conv2 = nn.Conv2d(64, 64, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.fc1 = nn.Linear(64 * 5 * 5, 384)
        self.fc2 = nn.Linear(384, 192)
        self.fc3 = nn.Linear(192, self.n_cls)

    def forward(self, x):
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = F.relu(self.fc1(x.flatten(1)))
        return self.fc3(F.relu(self.fc2(x)))


class cnn_cifar100(cnn_cifar10):
    n_cls = 100


class CNN_OriginalFedAvg(nn.Module):
    """FedAvg-paper EMNIST CNN (``cnn.py:6-72``)."""

    def __init__(self, only_digits=True):
        super().__init__()
        self.only_digits = only_digits
        self.conv2d_1 = nn.Conv2d(1, 32, 5, padding=2)
        self.max_pooling = nn.MaxPool2d(2, stride=2)
        self.conv2d_2 = nn.Conv2d(32, 64, 5, padding=2)
        self.flatten = nn.Flatten()
        self.linear_1 = nn.Linear(3136, 512)
        self.linear_2 = nn.Linear(512, 10 if only_digits else 62)
        self.relu = nn.ReLU()

    def forward(self, x):
        x = x.view(-1, 1, 28, 28)
        x = self.max_pooling(self.relu(self.conv2d_1(x)))
        x = self.max_pooling(self.relu(self.conv2d_2(x)))
        return self.linear_2(self.relu(self.linear_1(self.flatten(x))))


class CNN_DropOut(nn.Module):
    """EMNIST CNN with dropout (``cnn.py:75-142``)."""

    def __init__(self, only_digits=True):
        super().__init__()
        self.conv2d_1 = nn.Conv2d(1, 32, 3)
        self.max_pooling = nn.MaxPool2d(2, stride=2)
        self.conv2d_2 = nn.Conv2d(32, 64, 3)
        self.dropout_1 = nn.Dropout(0.25)
        self.flatten = nn.Flatten()
        self.linear_1 = nn.Linear(9216, 128)
        self.dropout_2 = nn.Dropout(0.5)
        self.linear_2 = nn.Linear(128, 10 if only_digits else 62)
        self.relu = nn.ReLU()

    def forward(self, x):
        x = x.view(-1, 1, 28, 28)
        x = self.relu(self.conv2d_1(x))
        x = self.dropout_1(self.max_pooling(self.relu(self.conv2d_2(x))))
        x = self.dropout_2(self.relu(self.linear_1(self.flatten(x))))
        return self.linear_2(x)


class cnn_cifar10_meta(nn.Module):
    """DisPFL-era CNN whose conv/fc layers are named ``*meta*`` for meta-mask experiments (``cnn_meta.py:17-120``):
    same topology as :class:`cnn_cifar10`; ``init_masks`` returns random masks for the meta layers."""

    def __init__(self, n_cls=10, dense_ratio=0.2):
        super().__init__()
        self.dense_ratio = dense_ratio
        self.conv1_meta = nn.Conv2d(3, 64, 5)
        self.conv2_meta = nn.Conv2d(64, 64, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.fc1_meta = nn.Linear(64 * 5 * 5, 384)
        self.fc2_meta = nn.Linear(384, 192)
        self.fc3 = nn.Linear(192, n_cls)

    def init_masks(self):
        return {name + ".weight": self.init_conv_masks(m.weight.shape, self.dense_ratio)
                for name, m in self.named_modules() if "meta" in name}

    @staticmethod
    def init_conv_masks(size, dense_ratio):
        mask = torch.zeros(size).view(-1)
        k = int(dense_ratio * mask.numel())
        if k > 0:
            mask[torch.randperm(mask.numel())[:k]] = 1
        return mask.view(size)

    def forward(self, x):
        x = self.pool(F.relu(self.conv1_meta(x)))
        x = self.pool(F.relu(self.conv2_meta(x)))
        x = F.relu(self.fc1_meta(x.flatten(1)))
        return self.fc3(F.relu(self.fc2_meta(x)))


class Meta_net(nn.Module):
    """Mask hypernetwork (``cnn_meta.py:123-177``): maps a layer's mask to a per-layer keep-score vector."""

    def __init__(self, mask):
        super().__init__()
        size = int(mask.flatten().shape[0])
        hid = max(1, int(math.sqrt(size)))
        self.fc11 = nn.Linear(size, hid)
        self.fc12 = nn.Linear(hid, hid)
        self.fc13 = nn.Linear(hid, size)

    def forward(self, x):
        return torch.sigmoid(self.fc13(F.relu(self.fc12(F.relu(self.fc11(x))))))


class LogisticRegression(nn.Module):
    """Multinomial / binary logistic regression on flat features (new; BASELINE.json config 1)."""

    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.linear = nn.Linear(input_dim, output_dim)

    def forward(self, x):
        return self.linear(x.flatten(1))
