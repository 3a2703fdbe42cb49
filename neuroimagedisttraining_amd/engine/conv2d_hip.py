"""Client-grouped layers for the batched 2-D image engine on the hand-written kernels (``conv2d_any.hip``).

The small models of the reference's entry points (``lenet5``, ``cnn_cifar10/100``, the EMNIST CNNs, ``vgg11/16`` —
``fedml_experiments/standalone/subavg/main_subavg.py:143-158``) run G clients of a lockstep step as one pass over
group-stacked tensors ``[G*B, C, H, W]``: a deep copy of the model whose ``Conv2d`` / ``Linear`` / ``GroupNorm``
modules are replaced by grouped twins reading the clients' parameter rows (``[G, *shape]`` views of theta):

* ``Conv2d`` (stride 1, any kernel size and channel count) -> :class:`HipConv2dFn`: forward and stride-1 data
  gradient on the implicit-GEMM MFMA kernel, weight gradient on the staged fp32 kernel (``conv2d_any.hip``); the
  activations stay channels-last (``torch.channels_last`` views), bf16;
* ``Linear`` -> one batched GEMM per layer (``baddbmm`` over the client axis);
* ``GroupNorm`` -> ``group_norm`` without affine on the stacked batch, then the per-client affine;
* everything else (ReLU, max-pool, dropout, flatten) is per-sample and runs unchanged on the stacked batch.

The model's own ``forward`` runs as written, so the layer order and every view/flatten are the reference's.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


_stream = ops.stream


def _nhwc_bf16(x):
    """[N, C, H, W]-shaped tensor -> contiguous channels-last bf16 [N, H, W, C] (no copy for a channels-last bf16
    input)."""
    t = x.permute(0, 2, 3, 1)
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t if t.is_contiguous() else t.contiguous()


def pack_conv_w(w):
    """fp32 [G, Cout, Cin, k, k] -> bf16 forward image [G, ceil64(Cout), k*k, ceil8(Cin)] (zero padded)."""
    G, co, ci, k, _ = w.shape
    img = w.permute(0, 1, 3, 4, 2).reshape(G, co, k * k, ci)
    img = F.pad(img, (0, (-ci) % 8, 0, 0, 0, (-co) % 64))
    return img.to(torch.bfloat16).contiguous()


def pack_conv_wt(w):
    """fp32 [G, Cout, Cin, k, k] -> the data-gradient image [G, ceil64(Cin), k*k, ceil8(Cout)]: the flipped kernel
    with input and output channels exchanged (dX = conv(dY, W^T flipped), padding k - 1 - p)."""
    G, co, ci, k, _ = w.shape
    img = w.flip(3, 4).permute(0, 2, 3, 4, 1).reshape(G, ci, k * k, co)
    img = F.pad(img, (0, (-co) % 8, 0, 0, 0, (-ci) % 64))
    return img.to(torch.bfloat16).contiguous()


class HipConv2dFn(torch.autograd.Function):
    """Grouped stride-1 conv: x [G*B, Cin, H, W] (any strides), w [G, Cout, Cin, k, k] fp32, b [G, Cout] or None."""

    @staticmethod
    def forward(ctx, x, w, b, G, pad):
        m = ops.ext()
        N, ci, H, W = x.shape
        co, k = w.shape[1], w.shape[3]
        assert N % G == 0 and w.shape[0] == G and w.shape[2] == ci
        B = N // G
        xs = _nhwc_bf16(x)
        Ho, Wo = H + 2 * pad - k + 1, W + 2 * pad - k + 1
        y = torch.empty(N, Ho, Wo, co, device=x.device, dtype=torch.bfloat16)
        wp = pack_conv_w(w.detach())
        bias = b.detach().float().contiguous() if b is not None else None
        m.conv2d_any_fwd(xs.data_ptr(), wp.data_ptr(), bias.data_ptr() if bias is not None else 0, y.data_ptr(), G, B,
                         H, W, ci, ci, co, k, pad, _stream())
        ctx.save_for_backward(xs, w)
        ctx.G, ctx.pad, ctx.has_b = G, pad, b is not None
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        m = ops.ext()
        xs, w = ctx.saved_tensors
        G, pad = ctx.G, ctx.pad
        N, H, W, ci = xs.shape
        co, k = w.shape[1], w.shape[3]
        B = N // G
        dy = _nhwc_bf16(gy)
        Ho, Wo = dy.shape[1], dy.shape[2]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wt = pack_conv_wt(w.detach())
            dxs = torch.empty(N, H, W, ci, device=xs.device, dtype=torch.bfloat16)
            m.conv2d_any_fwd(dy.data_ptr(), wt.data_ptr(), 0, dxs.data_ptr(), G, B, Ho, Wo, co, co, ci, k, k - 1 - pad,
                             _stream())
            dx = dxs.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            nch = m.conv2d_any_wgrad_chunks(B, Ho, Wo)
            part = torch.empty(nch, G, co, k * k, ci, device=xs.device, dtype=torch.float32)
            m.conv2d_any_wgrad(xs.data_ptr(), dy.data_ptr(), part.data_ptr(), G, B, H, W, ci, ci, co, k, pad,
                               _stream())
            dw = part.sum(0).view(G, co, k, k, ci).permute(0, 1, 4, 2, 3).contiguous()
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = dy.float().view(G, B * Ho * Wo, co).sum(1)
        return dx, dw, db, None, None


class _Group:
    """The current step's grouping: G and the per-client parameter views {name: [G, *shape]}."""

    def __init__(self):
        self.G = 1
        self.params = {}


class GConv2d(nn.Module):
    def __init__(self, mod, name, grp):
        super().__init__()
        assert mod.stride == (1, 1) and mod.dilation == (1, 1) and mod.groups == 1, "GConv2d: stride-1 plain convs"
        assert mod.kernel_size[0] == mod.kernel_size[1] and mod.padding[0] == mod.padding[1]
        self.name, self.grp, self.pad = name, grp, int(mod.padding[0])
        self.has_b = mod.bias is not None

    def forward(self, x):
        P = self.grp.params
        w, b = P[self.name + ".weight"], (P[self.name + ".bias"] if self.has_b else None)
        if not x.is_cuda:  # CPU twin (tests of the grouped graph): one grouped library conv over the client axis
            G = self.grp.G
            N, C, H, W = x.shape
            xc = x.reshape(G, N // G, C, H, W).transpose(0, 1).reshape(N // G, G * C, H, W)
            y = F.conv2d(xc, w.reshape((-1,) + tuple(w.shape[2:])), b.reshape(-1) if b is not None else None,
                         padding=self.pad, groups=G)
            return y.view(N // G, G, -1, *y.shape[2:]).transpose(0, 1).reshape(N, -1, *y.shape[2:])
        return HipConv2dFn.apply(x, w, b, self.grp.G, self.pad)


class GLinear(nn.Module):
    def __init__(self, mod, name, grp):
        super().__init__()
        self.name, self.grp, self.has_b = name, grp, mod.bias is not None

    def forward(self, x):
        G, P = self.grp.G, self.grp.params
        w = P[self.name + ".weight"]
        xg = x.reshape(G, x.shape[0] // G, x.shape[1])
        if not torch.is_autocast_enabled():
            xg = xg.to(w.dtype)
        if self.has_b:
            y = torch.baddbmm(P[self.name + ".bias"].unsqueeze(1), xg, w.transpose(1, 2))
        else:
            y = torch.bmm(xg, w.transpose(1, 2))
        return y.reshape(x.shape[0], w.shape[1])


class GGroupNorm(nn.Module):
    def __init__(self, mod, name, grp):
        super().__init__()
        self.name, self.grp = name, grp
        self.num_groups, self.eps, self.affine = mod.num_groups, mod.eps, mod.affine

    def forward(self, x):
        G = self.grp.G
        y = F.group_norm(x, self.num_groups, None, None, self.eps)
        if not self.affine:
            return y
        P = self.grp.params
        N, C = y.shape[:2]
        w = P[self.name + ".weight"].view((G, 1, C) + (1,) * (y.dim() - 2))
        b = P[self.name + ".bias"].view((G, 1, C) + (1,) * (y.dim() - 2))
        return (y.view((G, N // G) + tuple(y.shape[1:])) * w + b).view(y.shape)


_SWAP = {nn.Conv2d: GConv2d, nn.Linear: GLinear, nn.GroupNorm: GGroupNorm}


def supports(model):
    """True when every parametrised layer has a grouped twin (stride-1 plain Conv2d, Linear, GroupNorm)."""
    for mod in model.modules():
        if isinstance(mod, nn.Conv2d):
            if mod.stride != (1, 1) or mod.dilation != (1, 1) or mod.groups != 1 or \
                    mod.kernel_size[0] != mod.kernel_size[1] or mod.padding[0] != mod.padding[1] or \
                    mod.padding_mode != "zeros":
                return False
        elif len(list(mod.parameters(recurse=False))) and type(mod) not in _SWAP:
            return False
    return True


def grouped_model(model):
    """(deep copy of ``model`` with the grouped twins swapped in, its _Group holder)."""
    grp = _Group()
    gm = copy.deepcopy(model)

    def swap(parent, prefix):
        for cname, child in list(parent.named_children()):
            full = prefix + cname
            cls = _SWAP.get(type(child))
            if cls is not None:
                setattr(parent, cname, cls(child, full, grp))
            else:
                swap(child, full + ".")
    swap(gm, "")
    for p in gm.parameters():  # the twins read the clients' rows; no module parameters are left
        raise AssertionError("grouped_model: parameter left in the grouped copy")
    return gm, grp
