"""Evaluation networks built from a genotype (reference ``fedml_api/model/cv/darts/model.py:8-216``)."""
from __future__ import annotations

import torch
import torch.nn as nn

from .ops import OPS, FactorizedReduce, Identity, ReLUConvBN
from .utils import drop_path


class Cell(nn.Module):
    def __init__(self, genotype, C_prev_prev, C_prev, C, reduction, reduction_prev):
        super().__init__()
        self.reduction = reduction
        self.preprocess0 = FactorizedReduce(C_prev_prev, C) if reduction_prev else ReLUConvBN(C_prev_prev, C, 1, 1, 0)
        self.preprocess1 = ReLUConvBN(C_prev, C, 1, 1, 0)
        edges = genotype.reduce if reduction else genotype.normal
        self._concat = list(genotype.reduce_concat if reduction else genotype.normal_concat)
        self.multiplier = len(self._concat)
        self._steps = len(edges) // 2
        self._indices = [j for _, j in edges]
        self._ops = nn.ModuleList(OPS[name](C, 2 if reduction and j < 2 else 1, True) for name, j in edges)

    def forward(self, s0, s1, drop_prob=0.0):
        states = [self.preprocess0(s0), self.preprocess1(s1)]
        for i in range(self._steps):
            out = []
            for e in (2 * i, 2 * i + 1):
                h = self._ops[e](states[self._indices[e]])
                if self.training and drop_prob > 0.0 and not isinstance(self._ops[e], Identity):
                    h = drop_path(h, drop_prob)
                out.append(h)
            states.append(out[0] + out[1])
        return torch.cat([states[i] for i in self._concat], dim=1)


def _aux_features(C, pool_stride, with_last_bn):
    layers = [nn.ReLU(inplace=True), nn.AvgPool2d(5, stride=pool_stride, padding=0, count_include_pad=False),
              nn.Conv2d(C, 128, 1, bias=False), nn.BatchNorm2d(128), nn.ReLU(inplace=True),
              nn.Conv2d(128, 768, 2, bias=False)]
    if with_last_bn:
        layers.append(nn.BatchNorm2d(768))
    layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


class AuxiliaryHeadCIFAR(nn.Module):
    """Auxiliary classifier on an 8x8 feature map."""

    def __init__(self, C, num_classes):
        super().__init__()
        self.features = _aux_features(C, 3, True)
        self.classifier = nn.Linear(768, num_classes)

    def forward(self, x):
        return self.classifier(self.features(x).flatten(1))


class AuxiliaryHeadImageNet(nn.Module):
    """Auxiliary classifier on a 14x14 feature map (no BN after the 2x2 conv, as in the paper's runs)."""

    def __init__(self, C, num_classes):
        super().__init__()
        self.features = _aux_features(C, 2, False)
        self.classifier = nn.Linear(768, num_classes)

    def forward(self, x):
        return self.classifier(self.features(x).flatten(1))


def _stack_cells(owner, genotype, layers, C_pp, C_p, C, reduction_prev):
    owner.cells = nn.ModuleList()
    C_aux = None
    for i in range(layers):
        reduction = i in (layers // 3, 2 * layers // 3)
        if reduction:
            C *= 2
        cell = Cell(genotype, C_pp, C_p, C, reduction, reduction_prev)
        owner.cells.append(cell)
        reduction_prev = reduction
        C_pp, C_p = C_p, cell.multiplier * C
        if i == 2 * layers // 3:
            C_aux = C_p
    return C_p, C_aux


class _EvalNet(nn.Module):
    def _run_cells(self, s0, s1):
        aux = None
        for i, cell in enumerate(self.cells):
            s0, s1 = s1, cell(s0, s1, self.drop_path_prob)
            if i == 2 * self._layers // 3 and self._auxiliary and self.training:
                aux = self.auxiliary_head(s1)
        return s1, aux


class NetworkCIFAR(_EvalNet):
    def __init__(self, C, num_classes, layers, auxiliary, genotype, in_channels=3):
        super().__init__()
        self._layers, self._auxiliary = layers, auxiliary
        self.drop_path_prob = 0.5
        Cs = 3 * C
        self.stem = nn.Sequential(nn.Conv2d(in_channels, Cs, 3, padding=1, bias=False), nn.BatchNorm2d(Cs))
        C_prev, C_aux = _stack_cells(self, genotype, layers, Cs, Cs, C, False)
        if auxiliary:
            self.auxiliary_head = AuxiliaryHeadCIFAR(C_aux, num_classes)
        self.global_pooling = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(C_prev, num_classes)

    def forward(self, x):
        s = self.stem(x)
        s1, aux = self._run_cells(s, s)
        return self.classifier(self.global_pooling(s1).flatten(1)), aux


class NetworkImageNet(_EvalNet):
    def __init__(self, C, num_classes, layers, auxiliary, genotype, in_channels=3):
        super().__init__()
        self._layers, self._auxiliary = layers, auxiliary
        self.drop_path_prob = 0.5
        self.stem0 = nn.Sequential(nn.Conv2d(in_channels, C // 2, 3, stride=2, padding=1, bias=False),
                                   nn.BatchNorm2d(C // 2), nn.ReLU(inplace=True),
                                   nn.Conv2d(C // 2, C, 3, stride=2, padding=1, bias=False), nn.BatchNorm2d(C))
        self.stem1 = nn.Sequential(nn.ReLU(inplace=True), nn.Conv2d(C, C, 3, stride=2, padding=1, bias=False),
                                   nn.BatchNorm2d(C))
        C_prev, C_aux = _stack_cells(self, genotype, layers, C, C, C, True)
        if auxiliary:
            self.auxiliary_head = AuxiliaryHeadImageNet(C_aux, num_classes)
        self.global_pooling = nn.AvgPool2d(7)
        self.classifier = nn.Linear(C_prev, num_classes)

    def forward(self, x):
        s0 = self.stem0(x)
        s1, aux = self._run_cells(s0, self.stem1(s0))
        return self.classifier(self.global_pooling(s1).flatten(1)), aux
