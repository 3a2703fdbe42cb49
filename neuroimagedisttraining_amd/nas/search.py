"""DARTS / GDAS search networks (reference ``darts/model_search.py:10-306``, ``darts/model_search_gdas.py:9-188``).

* :class:`Network` — continuous relaxation: every edge is a softmax(alpha)-weighted sum of all 8 primitives.
* :class:`Network_GumbelSoftmax` — GDAS: hard Gumbel-softmax sample per edge; only ops with a non-zero
  (one-hot) weight are evaluated, but the straight-through weight keeps the gradient path to alpha.
* :func:`derive_genotype` — top-2 incoming edges per node by strongest non-'none' op, as the reference
  ``genotype()``; returns ``(Genotype, n_conv_normal, n_conv_reduce)`` (ops with index >= 4 are convs).
* :class:`ModelForModelSizeMeasure` — the argmax-discretised search network (used only for its size).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .genotypes import Genotype
from .ops import OPS, PRIMITIVES, FactorizedReduce, ReLUConvBN, search_op
from .utils import count_parameters_in_MB


def n_edges(steps):
    return sum(2 + i for i in range(steps))


class MixedOp(nn.Module):
    def __init__(self, C, stride):
        super().__init__()
        self._ops = nn.ModuleList(search_op(p, C, stride) for p in PRIMITIVES)

    def forward(self, x, weights, active=None):
        if active is None:
            return sum(w * op(x) for w, op in zip(weights, self._ops))
        terms = [weights[j] * self._ops[j](x) for j in active]
        return terms[0] if len(terms) == 1 else sum(terms)


class _SearchCellBase(nn.Module):
    def __init__(self, steps, multiplier, C_prev_prev, C_prev, C, reduction, reduction_prev):
        super().__init__()
        self.reduction = reduction
        self.preprocess0 = (FactorizedReduce(C_prev_prev, C, affine=False) if reduction_prev
                            else ReLUConvBN(C_prev_prev, C, 1, 1, 0, affine=False))
        self.preprocess1 = ReLUConvBN(C_prev, C, 1, 1, 0, affine=False)
        self._steps = steps
        self._multiplier = multiplier


class Cell(_SearchCellBase):
    def __init__(self, steps, multiplier, C_prev_prev, C_prev, C, reduction, reduction_prev):
        super().__init__(steps, multiplier, C_prev_prev, C_prev, C, reduction, reduction_prev)
        self._ops = nn.ModuleList(MixedOp(C, 2 if reduction and j < 2 else 1)
                                  for i in range(steps) for j in range(2 + i))

    def forward(self, s0, s1, weights, hard=False):
        states = [self.preprocess0(s0), self.preprocess1(s1)]
        active = None
        if hard:  # one host sync per cell (GDAS); picks the evaluated ops per edge
            nz = (weights.detach().abs() > 1e-10).cpu().tolist()
            active = [[k for k, b in enumerate(row) if b] for row in nz]
        off = 0
        for _ in range(self._steps):
            s = sum(self._ops[off + j](h, weights[off + j], None if active is None else active[off + j])
                    for j, h in enumerate(states))
            off += len(states)
            states.append(s)
        return torch.cat(states[-self._multiplier:], dim=1)


def _build_cells(owner, C, layers, steps, multiplier, stem_multiplier, cell_fn, in_ch=3):
    C_curr = stem_multiplier * C
    owner.stem = nn.Sequential(nn.Conv2d(in_ch, C_curr, 3, padding=1, bias=False), nn.BatchNorm2d(C_curr))
    C_prev_prev, C_prev, C_curr = C_curr, C_curr, C
    owner.cells = nn.ModuleList()
    reduction_prev = False
    for i in range(layers):
        reduction = i in (layers // 3, 2 * layers // 3)
        if reduction:
            C_curr *= 2
        owner.cells.append(cell_fn(C_prev_prev, C_prev, C_curr, reduction, reduction_prev))
        reduction_prev = reduction
        C_prev_prev, C_prev = C_prev, multiplier * C_curr
    owner.global_pooling = nn.AdaptiveAvgPool2d(1)
    return C_prev


def _parse_alpha(w, steps):
    """Top-2 input edges per node and their best non-'none' op."""
    none = PRIMITIVES.index("none")
    gene, n_conv, start = [], 0, 0
    for i in range(steps):
        W = w[start:start + i + 2]
        best = [max((k for k in range(W.shape[1]) if k != none), key=lambda k, r=r: W[r][k]) for r in range(i + 2)]
        edges = sorted(range(i + 2), key=lambda r: -W[r][best[r]])[:2]
        for j in edges:
            n_conv += int(best[j] >= 4)
            gene.append((PRIMITIVES[best[j]], j))
        start += i + 2
    return gene, n_conv


def derive_genotype(alphas_normal, alphas_reduce, steps=4, multiplier=4):
    with torch.no_grad():
        gn, cn = _parse_alpha(F.softmax(alphas_normal.float(), dim=-1).cpu().numpy(), steps)
        gr, cr = _parse_alpha(F.softmax(alphas_reduce.float(), dim=-1).cpu().numpy(), steps)
    concat = list(range(2 + steps - multiplier, steps + 2))
    return Genotype(normal=gn, normal_concat=concat, reduce=gr, reduce_concat=concat), cn, cr


class Network(nn.Module):
    """DARTS supernet.  ``forward`` returns logits; ``arch_parameters()`` = [alphas_normal, alphas_reduce]."""

    hard = False

    def __init__(self, C, num_classes, layers, criterion, device=None, steps=4, multiplier=4, stem_multiplier=3,
                 in_channels=3):
        super().__init__()
        self._C, self._num_classes, self._layers = C, num_classes, layers
        self._criterion = criterion
        self._steps, self._multiplier, self._stem_multiplier = steps, multiplier, stem_multiplier
        self._in_channels = in_channels
        self.device = device
        C_prev = _build_cells(self, C, layers, steps, multiplier, stem_multiplier,
                              lambda a, b, c, r, rp: Cell(steps, multiplier, a, b, c, r, rp), in_channels)
        self.classifier = nn.Linear(C_prev, num_classes)
        self._initialize_alphas()

    def _initialize_alphas(self):
        k, n = n_edges(self._steps), len(PRIMITIVES)
        self.alphas_normal = nn.Parameter(1e-3 * torch.randn(k, n))
        self.alphas_reduce = nn.Parameter(1e-3 * torch.randn(k, n))
        self._arch_parameters = [self.alphas_normal, self.alphas_reduce]

    def new(self):
        m = type(self)(self._C, self._num_classes, self._layers, self._criterion, self.device, self._steps,
                       self._multiplier, self._stem_multiplier, self._in_channels)
        if self.device is not None:
            m = m.to(self.device)
        with torch.no_grad():
            for x, y in zip(m.arch_parameters(), self.arch_parameters()):
                x.copy_(y)
        return m

    def new_arch_parameters(self):
        k, n = n_edges(self._steps), len(PRIMITIVES)
        dev = self.alphas_normal.device
        return [nn.Parameter(1e-3 * torch.randn(k, n, device=dev)), nn.Parameter(1e-3 * torch.randn(k, n, device=dev))]

    def arch_parameters(self):
        return self._arch_parameters

    def weight_parameters(self):
        ids = {id(p) for p in self._arch_parameters}
        return [p for p in self.parameters() if id(p) not in ids]

    def _edge_weights(self, alpha):
        return F.softmax(alpha, dim=-1)

    def forward(self, x):
        s0 = s1 = self.stem(x)
        wn = self._edge_weights(self.alphas_normal)
        wr = self._edge_weights(self.alphas_reduce)
        for cell in self.cells:
            s0, s1 = s1, cell(s0, s1, wr if cell.reduction else wn, self.hard)
        return self.classifier(self.global_pooling(s1).flatten(1))

    def loss(self, x, target):
        return self._criterion(self(x), target)

    def genotype(self):
        return derive_genotype(self.alphas_normal, self.alphas_reduce, self._steps, self._multiplier)

    def get_current_model_size(self):
        m = ModelForModelSizeMeasure(self._C, self._num_classes, self._layers, self._criterion, self.alphas_normal,
                                     self.alphas_reduce, self._steps, self._multiplier, self._stem_multiplier,
                                     self._in_channels)
        return count_parameters_in_MB(m)


class Network_GumbelSoftmax(Network):  # noqa: N801 (reference name)
    """GDAS supernet: hard straight-through Gumbel-softmax edge weights with temperature ``tau``."""

    hard = True

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.tau = 5.0

    def set_tau(self, tau):
        self.tau = tau

    def get_tau(self):
        return self.tau

    def _edge_weights(self, alpha):
        return F.gumbel_softmax(alpha, self.tau, hard=True)


class _ArgmaxCell(_SearchCellBase):
    def __init__(self, steps, multiplier, C_prev_prev, C_prev, C, reduction, reduction_prev, alphas):
        super().__init__(steps, multiplier, C_prev_prev, C_prev, C, reduction, reduction_prev)
        choice = alphas.detach().argmax(dim=-1).tolist()
        self._ops = nn.ModuleList()
        e = 0
        for i in range(steps):
            for j in range(2 + i):
                self._ops.append(search_op(PRIMITIVES[choice[e]], C, 2 if reduction and j < 2 else 1))
                e += 1

    def forward(self, s0, s1):
        states = [self.preprocess0(s0), self.preprocess1(s1)]
        off = 0
        for _ in range(self._steps):
            s = sum(self._ops[off + j](h) for j, h in enumerate(states))
            off += len(states)
            states.append(s)
        return torch.cat(states[-self._multiplier:], dim=1)


class ModelForModelSizeMeasure(nn.Module):
    """Search network with every edge fixed to its argmax op (reference ``model_search.py:106-170``).

    The reference maps the argmax index through ``OPS.keys()`` order (avg/max pool swapped relative to
    PRIMITIVES); both pools are parameter-free, so the measured size is identical."""

    def __init__(self, C, num_classes, layers, criterion, alphas_normal, alphas_reduce, steps=4, multiplier=4,
                 stem_multiplier=3, in_channels=3):
        super().__init__()
        self._criterion = criterion
        C_prev = _build_cells(self, C, layers, steps, multiplier, stem_multiplier,
                              lambda a, b, c, r, rp: _ArgmaxCell(steps, multiplier, a, b, c, r, rp,
                                                                 alphas_reduce if r else alphas_normal), in_channels)
        self.classifier = nn.Linear(C_prev, num_classes)

    def forward(self, x):
        s0 = s1 = self.stem(x)
        for cell in self.cells:
            s0, s1 = s1, cell(s0, s1)
        return self.classifier(self.global_pooling(s1).flatten(1))
