"""GroupNorm building blocks, ImageNet-style GroupNorm ResNets, synchronized BatchNorm and the
"global + personal" ResNet_ip.

Reference counterparts: ``group_normalization.py:7-118`` (GroupNorm2d/3d implemented through a reshaped
``F.batch_norm``), ``resnet_gn.py:20-235`` (ResNet-18..152 with GroupNorm), ``batchnorm_utils.py:150-463``
(SynchronizedBatchNorm{1,2,3}d over ``nn.DataParallel``) and ``resnet_ip.py:33-359``.

MI355X design: synchronized BN here is one process per GPU — the per-channel (sum, sum of squares, count)
vector is all-reduced over RCCL (``torch.distributed``, backend "nccl") in the forward and the (dy, dy*xhat)
sums in the backward; without an initialised process group it is plain BatchNorm.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class _GroupNormNd(nn.Module):
    """GroupNorm computed as batch-norm over (N*G) "channels" — same math as ``F.group_norm``."""

    def __init__(self, num_features, num_groups=32, eps=1e-5, affine=True):
        super().__init__()
        if num_features % num_groups:
            raise ValueError("num_features must be divisible by num_groups")
        self.num_features, self.num_groups, self.eps, self.affine = num_features, num_groups, eps, affine
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x):
        n = x.shape[0]
        y = x.reshape(1, n * self.num_groups, -1)
        y = F.batch_norm(y, None, None, training=True, eps=self.eps).view_as(x)
        if self.affine:
            shape = (1, -1) + (1,) * (x.dim() - 2)
            y = y * self.weight.view(shape) + self.bias.view(shape)
        return y


class GroupNorm2d(_GroupNormNd):
    pass


class GroupNorm3d(_GroupNormNd):
    pass


# ------------------------------------------------------------------------------------------------
def _gn(c, groups=32):
    return GroupNorm2d(c, groups)


class GNBasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=32):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = _gn(planes, groups)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = _gn(planes, groups)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        return self.relu(self.bn2(self.conv2(y)) + idt)


class GNBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=32):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _gn(planes, groups)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = _gn(planes, groups)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _gn(planes * 4, groups)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + idt)


class ResNetGN(nn.Module):
    """ImageNet-style ResNet (7x7 stem) with GroupNorm2d (``resnet_gn.py``)."""

    def __init__(self, block, layers, num_classes=1000, groups=32):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = _gn(64, groups)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0], 1, groups)
        self.layer2 = self._make(block, 128, layers[1], 2, groups)
        self.layer3 = self._make(block, 256, layers[2], 2, groups)
        self.layer4 = self._make(block, 512, layers[3], 2, groups)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make(self, block, planes, n, stride, groups):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 _gn(planes * block.expansion, groups))
        layers = [block(self.inplanes, planes, stride, down, groups)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, groups=groups) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(self.avgpool(x).flatten(1))


def resnet18_gn(num_classes=1000, **kw):
    return ResNetGN(GNBasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34_gn(num_classes=1000, **kw):
    return ResNetGN(GNBasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50_gn(num_classes=1000, **kw):
    return ResNetGN(GNBottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101_gn(num_classes=1000, **kw):
    return ResNetGN(GNBottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152_gn(num_classes=1000, **kw):
    return ResNetGN(GNBottleneck, [3, 8, 36, 3], num_classes, **kw)


# ------------------------------------------------------------------------------------------------
class _SyncBNFn(torch.autograd.Function):
    """Cross-process BatchNorm statistics over RCCL: one all-reduce of [sum, sumsq, count] per forward and one
    of [sum dy, sum dy*xhat] per backward (reference: ReduceAddCoalesced/Broadcast, batchnorm_utils.py:214,217)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, group):
        c = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xf = x.float()
        stats = torch.cat([xf.sum(dims), (xf * xf).sum(dims),
                           torch.full((1,), float(x.numel() // c), device=x.device)])
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(stats, group=group)
        n = stats[-1]
        mean = stats[:c] / n
        var = (stats[c:2 * c] / n - mean * mean).clamp_min(0)
        invstd = torch.rsqrt(var + eps)
        shape = (1, -1) + (1,) * (x.dim() - 2)
        xhat = (xf - mean.view(shape)) * invstd.view(shape)
        y = xhat * weight.view(shape) + bias.view(shape)
        ctx.save_for_backward(xhat, weight, invstd, n)
        ctx.group = group
        ctx.shape = shape
        ctx.dims = dims
        return y.to(x.dtype), mean, var * n / (n - 1).clamp_min(1)

    @staticmethod
    def backward(ctx, dy, _dm, _dv):
        xhat, weight, invstd, n = ctx.saved_tensors
        dyf = dy.float()
        c = xhat.shape[1]
        sums = torch.cat([dyf.sum(ctx.dims), (dyf * xhat).sum(ctx.dims)])
        dbias, dweight = sums[:c].clone(), sums[c:].clone()
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(sums, group=ctx.group)
        s = ctx.shape
        dx = (weight * invstd).view(s) * (dyf - (sums[:c] / n).view(s) - xhat * (sums[c:] / n).view(s))
        return dx.to(dy.dtype), dweight, dbias, None, None


class _SynchronizedBatchNorm(nn.BatchNorm1d):
    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, process_group=None):
        super().__init__(num_features, eps, momentum, affine)
        self.process_group = process_group

    def forward(self, x):
        if not self.training:
            return super().forward(x)
        w = self.weight if self.affine else torch.ones(self.num_features, device=x.device)
        b = self.bias if self.affine else torch.zeros(self.num_features, device=x.device)
        y, mean, var_unbiased = _SyncBNFn.apply(x, w, b, self.eps, self.process_group)
        with torch.no_grad():
            self.running_mean.mul_(1 - self.momentum).add_(mean.detach(), alpha=self.momentum)
            self.running_var.mul_(1 - self.momentum).add_(var_unbiased.detach(), alpha=self.momentum)
            self.num_batches_tracked += 1
        return y


class SynchronizedBatchNorm1d(_SynchronizedBatchNorm):
    pass


class SynchronizedBatchNorm2d(_SynchronizedBatchNorm):
    pass


class SynchronizedBatchNorm3d(_SynchronizedBatchNorm):
    pass


def convert_sync_batchnorm(module, process_group=None):
    """Replace every BatchNorm{1,2,3}d with its RCCL-synchronised counterpart (weights/buffers copied)."""
    out = module
    mapping = {nn.BatchNorm1d: SynchronizedBatchNorm1d, nn.BatchNorm2d: SynchronizedBatchNorm2d,
               nn.BatchNorm3d: SynchronizedBatchNorm3d}
    if type(module) in mapping:
        out = mapping[type(module)](module.num_features, module.eps, module.momentum or 0.1, module.affine,
                                    process_group)
        if module.affine:
            out.weight.data.copy_(module.weight.data)
            out.bias.data.copy_(module.bias.data)
        out.running_mean.copy_(module.running_mean)
        out.running_var.copy_(module.running_var)
        out.num_batches_tracked.copy_(module.num_batches_tracked)
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, process_group))
    return out


# ------------------------------------------------------------------------------------------------
class IPConv2d(nn.Module):
    """Convolution whose effective kernel is ``conv_g.weight + conv_v.weight`` (global + personal parts)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv_g = nn.Conv2d(cin, cout, k, stride, padding, bias=False)
        self.conv_v = nn.Conv2d(cin, cout, k, stride, padding, bias=False)
        nn.init.zeros_(self.conv_v.weight)
        self.stride, self.padding = stride, padding

    def forward(self, x):
        return F.conv2d(x, self.conv_g.weight + self.conv_v.weight, None, self.stride, self.padding)


class IPBlock(nn.Module):
    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = IPConv2d(cin, cout, 3, stride, 1)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = IPConv2d(cout, cout, 3, 1, 1)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + (x if self.shortcut is None else self.shortcut(x)))


class ResNet_ip(nn.Module):
    """CIFAR ResNet-{20,29,56,110}-style network with global+personal summed kernels (``resnet_ip.py:33-359``)."""

    def __init__(self, depth=56, num_classes=10):
        super().__init__()
        n = (depth - 2) // 6
        self.conv1 = IPConv2d(3, 16, 3, 1, 1)
        self.bn1 = nn.BatchNorm2d(16)
        layers, cin = [], 16
        for i, c in enumerate((16, 32, 64)):
            for j in range(n):
                layers.append(IPBlock(cin, c, 2 if (j == 0 and i > 0) else 1))
                cin = c
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(64, num_classes)

    def global_params(self):
        return {k: v for k, v in self.named_parameters() if "conv_v" not in k}

    def personal_params(self):
        return {k: v for k, v in self.named_parameters() if "conv_v" in k}

    def forward(self, x):
        x = self.layers(F.relu(self.bn1(self.conv1(x))))
        return self.fc(F.adaptive_avg_pool2d(x, 1).flatten(1))


def resnet29_ip(num_classes=10):
    return ResNet_ip(29, num_classes)


def resnet56_ip(num_classes=10):
    return ResNet_ip(56, num_classes)


def resnet110_ip(num_classes=10):
    return ResNet_ip(110, num_classes)


def DataParallelWithCallback(module, device_ids=None, output_device=None):  # noqa: N802 (reference name)
    """Reference ``batchnorm_utils.DataParallelWithCallback`` (single-process ``nn.DataParallel`` whose replicas
    sync BN through a master callback).  MI355X-native equivalent: one process per GPU — when a process group
    is initialised the module is wrapped in ``DistributedDataParallel`` (gradients all-reduced over RCCL,
    :class:`SynchronizedBatchNorm2d` statistics all-reduced in its forward); otherwise it is returned as is."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dev = next(module.parameters()).device
        ids = [dev.index] if dev.type == "cuda" else None
        return torch.nn.parallel.DistributedDataParallel(module, device_ids=ids, output_device=output_device)
    return module


def patch_replication_callback(data_parallel):
    """No-op: there are no in-process replicas to patch (see :func:`DataParallelWithCallback`)."""
    return data_parallel
