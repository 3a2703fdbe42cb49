"""DARTS candidate operations (reference ``fedml_api/model/cv/darts/operations.py:1-107``).

Same op set, same module structure (so state_dict keys and parameter counts match the reference), written
as small builders.  On MI355X these 2D ops run through MIOpen; the search/eval networks are used with
``channels_last`` memory format and bf16 autocast by :mod:`neuroimagedisttraining_amd.nas.train`.
"""
from __future__ import annotations

import torch
import torch.nn as nn

PRIMITIVES = ["none", "max_pool_3x3", "avg_pool_3x3", "skip_connect",
              "sep_conv_3x3", "sep_conv_5x5", "dil_conv_3x3", "dil_conv_5x5"]


def _relu_conv_bn(cin, cout, k, stride, pad, affine, dilation=1, groups=1):
    return [nn.ReLU(inplace=False),
            nn.Conv2d(cin, cout, k, stride=stride, padding=pad, dilation=dilation, groups=groups, bias=False)]


class ReLUConvBN(nn.Module):
    """ReLU -> Conv(k, stride, pad) -> BN."""

    def __init__(self, C_in, C_out, kernel_size, stride, padding, affine=True):
        super().__init__()
        self.op = nn.Sequential(*_relu_conv_bn(C_in, C_out, kernel_size, stride, padding, affine),
                                nn.BatchNorm2d(C_out, affine=affine))

    def forward(self, x):
        return self.op(x)


class DilConv(nn.Module):
    """ReLU -> depthwise dilated conv -> pointwise conv -> BN."""

    def __init__(self, C_in, C_out, kernel_size, stride, padding, dilation, affine=True):
        super().__init__()
        self.op = nn.Sequential(*_relu_conv_bn(C_in, C_in, kernel_size, stride, padding, affine, dilation, C_in),
                                nn.Conv2d(C_in, C_out, 1, bias=False), nn.BatchNorm2d(C_out, affine=affine))

    def forward(self, x):
        return self.op(x)


class SepConv(nn.Module):
    """Two stacked (ReLU, depthwise, pointwise, BN) blocks; only the first is strided."""

    def __init__(self, C_in, C_out, kernel_size, stride, padding, affine=True):
        super().__init__()
        layers = _relu_conv_bn(C_in, C_in, kernel_size, stride, padding, affine, 1, C_in)
        layers += [nn.Conv2d(C_in, C_in, 1, bias=False), nn.BatchNorm2d(C_in, affine=affine)]
        layers += _relu_conv_bn(C_in, C_in, kernel_size, 1, padding, affine, 1, C_in)
        layers += [nn.Conv2d(C_in, C_out, 1, bias=False), nn.BatchNorm2d(C_out, affine=affine)]
        self.op = nn.Sequential(*layers)

    def forward(self, x):
        return self.op(x)


class Identity(nn.Module):
    def forward(self, x):
        return x


class Zero(nn.Module):
    """The 'none' op: zeros of the (possibly strided) output shape."""

    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        if self.stride == 1:
            return x.mul(0.0)
        return x[:, :, ::self.stride, ::self.stride].mul(0.0)


class FactorizedReduce(nn.Module):
    """Stride-2 reduction by two 1x1 convs on offset grids, concatenated, then BN."""

    def __init__(self, C_in, C_out, affine=True):
        super().__init__()
        assert C_out % 2 == 0
        self.relu = nn.ReLU(inplace=False)
        self.conv_1 = nn.Conv2d(C_in, C_out // 2, 1, stride=2, bias=False)
        self.conv_2 = nn.Conv2d(C_in, C_out // 2, 1, stride=2, bias=False)
        self.bn = nn.BatchNorm2d(C_out, affine=affine)

    def forward(self, x):
        x = self.relu(x)
        return self.bn(torch.cat([self.conv_1(x), self.conv_2(x[:, :, 1:, 1:])], dim=1))


def _conv_7x1_1x7(C, stride, affine):
    return nn.Sequential(nn.ReLU(inplace=False),
                         nn.Conv2d(C, C, (1, 7), stride=(1, stride), padding=(0, 3), bias=False),
                         nn.Conv2d(C, C, (7, 1), stride=(stride, 1), padding=(3, 0), bias=False),
                         nn.BatchNorm2d(C, affine=affine))


OPS = {
    "none": lambda C, s, a: Zero(s),
    "avg_pool_3x3": lambda C, s, a: nn.AvgPool2d(3, stride=s, padding=1, count_include_pad=False),
    "max_pool_3x3": lambda C, s, a: nn.MaxPool2d(3, stride=s, padding=1),
    "skip_connect": lambda C, s, a: Identity() if s == 1 else FactorizedReduce(C, C, affine=a),
    "sep_conv_3x3": lambda C, s, a: SepConv(C, C, 3, s, 1, affine=a),
    "sep_conv_5x5": lambda C, s, a: SepConv(C, C, 5, s, 2, affine=a),
    "sep_conv_7x7": lambda C, s, a: SepConv(C, C, 7, s, 3, affine=a),
    "dil_conv_3x3": lambda C, s, a: DilConv(C, C, 3, s, 2, 2, affine=a),
    "dil_conv_5x5": lambda C, s, a: DilConv(C, C, 5, s, 4, 2, affine=a),
    "conv_7x1_1x7": _conv_7x1_1x7,
}


def search_op(primitive, C, stride):
    """Op as used inside a search-space MixedOp: affine-free, pools followed by a non-affine BN."""
    op = OPS[primitive](C, stride, False)
    if "pool" in primitive:
        op = nn.Sequential(op, nn.BatchNorm2d(C, affine=False))
    return op
