"""Flat, client-stacked parameter storage.

Every local client's model lives as one row of a ``[C, P]`` fp32 matrix (``P`` = parameters of one
model, 2,570,241 for AlexNet3D_Dropout).  Per-parameter tensors are views into that row
(``ParamLayout.view``), so fused multi-tensor kernels (clip + SGD + mask, aggregation, saliency,
top-k) touch a single contiguous buffer per client, and aggregation across clients/GPUs is a
single ``[C] x [C, P]`` contraction followed by one RCCL all-reduce of ``P`` floats.

Buffers (BN running stats, ``num_batches_tracked``) are stacked the same way in a separate
``[C, Q]`` fp32 matrix (the reference averages them too, quirk Q3).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field

import torch


@dataclass
class ParamLayout:
    names: list = field(default_factory=list)
    shapes: list = field(default_factory=list)
    offsets: list = field(default_factory=list)
    dtypes: list = field(default_factory=list)
    total: int = 0

    @classmethod
    def from_tensors(cls, named):
        lay = cls()
        off = 0
        for n, t in named:
            lay.names.append(n)
            lay.shapes.append(tuple(t.shape))
            lay.offsets.append(off)
            lay.dtypes.append(t.dtype)
            off += t.numel()
        lay.total = off
        return lay

    def index(self, name):
        return self.names.index(name)

    def numel(self, i):
        n = 1
        for d in self.shapes[i]:
            n *= d
        return n

    def view(self, flat, name):
        """``flat`` is ``[C, P]`` -> ``[C, *shape]`` view of parameter ``name``."""
        i = self.index(name)
        o, n = self.offsets[i], self.numel(i)
        return flat[:, o:o + n].view((flat.shape[0],) + self.shapes[i])

    def views(self, flat):
        return OrderedDict((n, self.view(flat, n)) for n in self.names)

    def flatten_state(self, sd, device=None, dtype=torch.float32):
        """state dict (single model) -> ``[P]`` vector."""
        parts = [sd[n].reshape(-1).to(device=device, dtype=dtype) for n in self.names]
        return torch.cat(parts) if parts else torch.zeros(0, device=device, dtype=dtype)

    def unflatten(self, vec):
        """``[P]`` vector -> OrderedDict of tensors with original dtypes (ints rounded)."""
        out = OrderedDict()
        for i, n in enumerate(self.names):
            t = vec[self.offsets[i]:self.offsets[i] + self.numel(i)].view(self.shapes[i])
            dt = self.dtypes[i]
            out[n] = t.clone() if dt.is_floating_point else t.round().to(dt)
        return out
