"""``nn.Module`` front-ends for the HIP kernels, so ordinary PyTorch models (not only the fused AlexNet3D engine)
run their hot 3D convolutions on the hand-written gfx950 kernels.

:class:`HipConv3d` is a drop-in ``nn.Conv3d`` (same parameters, same ``state_dict`` keys) for the 3x3x3,
stride-1, dilation-1, ungrouped convolutions with ``pad <= 2`` and channel counts that are multiples of 64
(<= 512) — in a 3D ResNet-50 that is 13 of the 16 bottleneck 3x3x3 convolutions (the stride-2 ones, the 7x7x7
stem and the 1x1x1 projections stay on MIOpen / hipBLASLt GEMMs).  On a CUDA (ROCm) tensor it routes through
``torch.ops.nidt.conv3d_k3`` (LDS-DMA implicit GEMM forward, dgrad on the flipped weights, row-group wgrad;
bf16 operands, fp32 accumulation and fp32 weight gradients); on CPU, or for an ineligible shape, it is exactly
``nn.Conv3d``.  The kernels are channels-last: an NCDHW input is transposed on the way in and the output is
returned in the caller's layout (with ``torch.channels_last_3d`` activations both transposes are free views).

Reference: ``fedml_api/model/cv/salient_models.py:8-139`` (3D ResNet blocks); BASELINE config 5.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def hip_conv_eligible(conv: nn.Conv3d) -> bool:
    k, s, d, p = conv.kernel_size, conv.stride, conv.dilation, conv.padding
    return (isinstance(conv, nn.Conv3d) and tuple(k) == (3, 3, 3) and tuple(s) == (1, 1, 1)
            and tuple(d) == (1, 1, 1) and conv.groups == 1 and isinstance(p, tuple) and len(set(p)) == 1
            and 0 <= p[0] <= 2 and conv.padding_mode == "zeros"
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0
            and conv.in_channels <= 512 and conv.out_channels <= 512)


class HipConv3d(nn.Conv3d):
    """``nn.Conv3d`` whose CUDA forward/backward run on ``nidt::conv3d_k3``."""

    def forward(self, x):
        if not (x.is_cuda and hip_conv_eligible(self)):
            return super().forward(x)
        from . import library  # noqa: F401  (registers torch.ops.nidt.*)
        pad = self.padding[0]
        xl = x.permute(0, 2, 3, 4, 1)  # NDHWC (a view when x is channels_last_3d)
        if xl.dtype != torch.bfloat16:
            xl = xl.to(torch.bfloat16)
        w = self.weight
        if w.dtype != torch.float32:
            w = w.float()
        bias = self.bias.float().view(1, -1) if self.bias is not None else \
            torch.zeros(1, self.out_channels, device=x.device, dtype=torch.float32)
        y = torch.ops.nidt.conv3d_k3(xl.contiguous(), w.unsqueeze(0), bias, pad)
        y = y.permute(0, 4, 1, 2, 3)  # NCDHW view with channels_last_3d strides
        if not x.is_contiguous(memory_format=torch.channels_last_3d):
            y = y.contiguous()  # follow the caller's layout (MIOpen's NDHWC batch norm is not used by default)
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype)


def use_hip_convs(model: nn.Module, channels_last: bool = False) -> int:
    """Swap every eligible ``nn.Conv3d`` of ``model`` for a :class:`HipConv3d` sharing its parameters (in place);
    returns the number swapped.  ``channels_last`` also moves the model to ``torch.channels_last_3d`` (saves the
    layout copies around each HIP conv; off by default: MIOpen's NDHWC 3D batch norm crashed on this image)."""
    n = 0
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if type(child) is nn.Conv3d and hip_conv_eligible(child):
                new = HipConv3d(child.in_channels, child.out_channels, child.kernel_size, child.stride,
                                child.padding, child.dilation, child.groups, child.bias is not None,
                                child.padding_mode, device=child.weight.device, dtype=child.weight.dtype)
                new.weight = child.weight
                if child.bias is not None:
                    new.bias = child.bias
                setattr(mod, cname, new)
                n += 1
    if channels_last:
        model.to(memory_format=torch.channels_last_3d)
    return n


def reference_conv3d(x, conv: nn.Conv3d):
    """fp32 PyTorch oracle of a (Hip)Conv3d forward (numerics tests)."""
    return F.conv3d(x.float(), conv.weight.float(), None if conv.bias is None else conv.bias.float(),
                    conv.stride, conv.padding, conv.dilation, conv.groups)
