"""Analytic FLOP counting (reference ``fedml_api/utils/main_flops_counter.py:30-163``).

Forward hooks count the FLOPs (2 per multiply-add) of Conv1d/2d/3d and Linear layers (sparse-aware: only non-zero weights unless
``full=True``); training = 3x inference (the reference's rule).  Unlike the reference (quirk Q15) Conv3d is
counted and each dataset uses its true input shape (ABCD: 1x121x145x121 rather than 1x32x32).
"""
from __future__ import annotations

import torch
import torch.nn as nn

INPUT_SHAPES = {"emnist": (1, 28, 28), "mnist": (1, 28, 28), "cifar10": (3, 32, 32), "cifar100": (3, 32, 32),
                "tiny": (3, 64, 64), "ABCD": (1, 121, 145, 121)}


def count_model_param_flops(model, dataset="ABCD", full=False, input_shape=None):
    """The reference counter with ``multiply_adds=True`` (its default, ``main_flops_counter.py:38``): a conv adds
    ``(2 * nnz(weight) + bias * Cout) * H_out * W_out`` (``:58-66``), a linear layer
    ``batch * (2 * nnz(weight) + nnz(bias))`` (``:71-80``; ``full`` counts every element instead of the non-zeros)."""
    counts = []

    def conv_hook(m, inp, out):
        nnz = m.weight.numel() if full else int(torch.count_nonzero(m.weight))
        bias = 1 if m.bias is not None else 0
        counts.append((2.0 * nnz / m.out_channels + bias) * out.numel())

    def linear_hook(m, inp, out):
        w = m.weight.numel() if full else int(torch.count_nonzero(m.weight))
        bias = 0 if m.bias is None else (m.bias.numel() if full else int(torch.count_nonzero(m.bias)))
        batch = out.numel() // m.out_features
        counts.append((2 * w + bias) * batch)

    handles = []
    for m in model.modules():
        if isinstance(m, (nn.Conv1d, nn.Conv2d, nn.Conv3d)):
            handles.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, nn.Linear):
            handles.append(m.register_forward_hook(linear_hook))
    shape = input_shape or INPUT_SHAPES.get(dataset, (3, 32, 32))
    dev = next(model.parameters()).device
    was = model.training
    model.eval()
    with torch.no_grad():
        model(torch.rand((1,) + tuple(shape), device=dev))
    model.train(was)
    for h in handles:
        h.remove()
    return float(sum(counts))


def count_inference_flops(model, dataset="ABCD", full=False, input_shape=None):
    return count_model_param_flops(model, dataset, full, input_shape)


def count_training_flops(model, dataset="ABCD", full=False, input_shape=None):
    return 3.0 * count_model_param_flops(model, dataset, full, input_shape)


def print_model_param_nums(model=None):
    """``main_flops_counter.py:24-28``: prints (and returns) the number of non-zero entries of the 4-D and 2-D
    parameters (2-D conv kernels and linear weights — the reference's rule, so 3-D conv kernels are not counted).
    The reference's default model is torchvision's AlexNet; torchvision is not a dependency here, so a model is
    required."""
    if model is None:
        raise ValueError("print_model_param_nums: pass a model (the torchvision AlexNet default is not available)")
    total = sum(int((p != 0).sum()) for p in model.parameters() if p.dim() in (2, 4))
    print('  + Number of params: %.2f' % (total))
    return total
