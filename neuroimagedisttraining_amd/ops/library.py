"""``torch.library`` custom ops over the gfx950 HIP kernels (namespace ``nidt``), with autograd.

These make the hand-written kernels usable from ordinary PyTorch code (any model, autograd, fake-tensor
shape propagation), not only from the fused AlexNet3D engine:

* ``nidt::conv3d_k3(x, w, bias, pad)`` — client-grouped 3x3x3 stride-1 Conv3d, channels-last:
  ``x [G*B, D, H, W, Cin]`` bf16, ``w [G, Cout, Cin, 3, 3, 3]`` fp32 (one weight set per client, PyTorch
  layout), ``bias [G, Cout]`` fp32 -> ``y [G*B, Do, Ho, Wo, Cout]`` bf16.  Forward = LDS-DMA implicit GEMM
  (``k_conv_fwd_dma``); backward: dX = the same kernel on flipped/transposed weights, dW = the row-group
  wgrad kernel (fp32, PyTorch layout), dbias = per-client channel sums.
* ``nidt::kth_largest(v, k)`` — radix select (k-th largest of a non-negative fp32 vector).
* ``nidt::weighted_rows_sum(rows, w)`` — ``sum_r w[r] * rows[r]`` (FedAvg aggregation kernel).

Host-side checks run before every launch (a mis-shaped launch can fault the GPU).  Reference: the ops the
reference runs through cuDNN/ATen (``salient_models.py:147-165``, ``snip.py:86-98``,
``sailentgrads_api.py:212-227``); SURVEY.md §7.1(a).
"""
from __future__ import annotations

import torch

from . import ext
from . import stream as _raw_stream

_LIB = "nidt"


_stream = _raw_stream


def _check_conv(x, w, bias, pad):
    if not (x.is_cuda and w.is_cuda and bias.is_cuda):
        raise ValueError("nidt::conv3d_k3 needs CUDA tensors")
    if x.dtype != torch.bfloat16 or w.dtype != torch.float32 or bias.dtype != torch.float32:
        raise TypeError("nidt::conv3d_k3: x bf16, w fp32, bias fp32")
    if x.dim() != 5 or w.dim() != 6 or tuple(w.shape[3:]) != (3, 3, 3):
        raise ValueError("nidt::conv3d_k3: x [G*B,D,H,W,Cin], w [G,Cout,Cin,3,3,3]")
    G, Cout, Cin = w.shape[:3]
    if x.shape[0] % G or x.shape[4] != Cin or tuple(bias.shape) != (G, Cout):
        raise ValueError("nidt::conv3d_k3: shape mismatch x%s w%s bias%s" % (tuple(x.shape), tuple(w.shape),
                                                                          tuple(bias.shape)))
    if Cin % 64 or Cin > 512 or Cout % 64 or Cout > 512:
        raise ValueError("nidt::conv3d_k3: Cin and Cout must be multiples of 64 and <= 512")
    if not 0 <= pad <= 2:
        raise ValueError("nidt::conv3d_k3: pad in [0, 2]")
    if any(s + 2 * pad - 2 <= 0 for s in x.shape[1:4]):
        raise ValueError("nidt::conv3d_k3: empty output")
    return G, x.shape[0] // G, Cin, Cout


def _pack(w, G, Cout, Cin, transposed):
    m = ext()
    flat = w.detach().reshape(G, -1).contiguous()
    wp = torch.empty(G, Cout, 27, Cin, device=w.device, dtype=torch.bfloat16)
    wt = torch.empty(G, Cin, 27, Cout, device=w.device, dtype=torch.bfloat16) if transposed else None
    m.pack_conv_w(flat.data_ptr(), flat.stride(0), 0, G, Cout, Cin, 1.0, wp.data_ptr(),
                  wt.data_ptr() if transposed else 0, _stream())
    return wp, wt


@torch.library.custom_op("nidt::conv3d_k3", mutates_args=())
def conv3d_k3(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, pad: int) -> torch.Tensor:
    G, B, Cin, Cout = _check_conv(x, w, bias, pad)
    x = x.contiguous()
    D, H, W = x.shape[1:4]
    wp, _ = _pack(w, G, Cout, Cin, False)
    y = torch.empty(G * B, D + 2 * pad - 2, H + 2 * pad - 2, W + 2 * pad - 2, Cout, device=x.device,
                    dtype=torch.bfloat16)
    b = bias.contiguous()
    ext().conv3d_fwd(x.data_ptr(), wp.data_ptr(), b.data_ptr(), 0, 0, y.data_ptr(), 0, G, B, D, H, W, Cin, Cout,
                     pad, _stream())
    return y


@conv3d_k3.register_fake
def _(x, w, bias, pad):
    D, H, W = x.shape[1:4]
    return x.new_empty((x.shape[0], D + 2 * pad - 2, H + 2 * pad - 2, W + 2 * pad - 2, w.shape[1]))


@torch.library.custom_op("nidt::conv3d_k3_backward", mutates_args=())
def conv3d_k3_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, pad: int,
                       need_dx: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    G, Cout, Cin = w.shape[:3]
    B = x.shape[0] // G
    D, H, W = x.shape[1:4]
    Do, Ho, Wo = dy.shape[1:4]
    m, st = ext(), _stream()
    dy = dy.contiguous().to(torch.bfloat16)
    x = x.contiguous()
    # dW: LDS-DMA row-group wgrad into fp32 PyTorch-layout rows
    K = 27 * Cin
    ns = m.conv3d_wgrad_nsplit(G, B, D, H, W, Cin, Cout, pad)
    part = torch.empty(ns * G * Cout * K, device=x.device, dtype=torch.float32)
    dw = torch.empty(G, Cout * K, device=x.device, dtype=torch.float32)
    ptab = torch.empty(B * Do * Ho * Wo, 2, device=x.device, dtype=torch.int32)
    m.conv3d_pos_table(ptab.data_ptr(), B, D, H, W, pad, st)
    m.conv3d_wgrad(x.data_ptr(), 0, 0, dy.data_ptr(), part.data_ptr(), dw.data_ptr(), dw.stride(0), 0, G, B, D, H,
                   W, Cin, Cout, pad, ns, 1.0, ptab.data_ptr(), st)
    db = dy.view(G, -1, Cout).float().sum(1)
    if need_dx:
        _, wt = _pack(w, G, Cout, Cin, True)
        dx = torch.empty_like(x)
        m.conv3d_fwd(dy.data_ptr(), wt.data_ptr(), 0, 0, 0, dx.data_ptr(), 0, G, B, Do, Ho, Wo, Cout, Cin, 2 - pad, st)
    else:
        dx = torch.zeros(0, device=x.device, dtype=x.dtype)
    return dx, dw.view_as(w), db


@conv3d_k3_backward.register_fake
def _(dy, x, w, pad, need_dx):
    dx = x.new_empty(x.shape) if need_dx else x.new_empty((0,))
    return dx, w.new_empty(w.shape), w.new_empty((w.shape[0], w.shape[1]))


def _setup(ctx, inputs, output):
    x, w, bias, pad = inputs
    ctx.save_for_backward(x, w)
    ctx.pad = pad


def _backward(ctx, dy):
    x, w = ctx.saved_tensors
    dx, dw, db = conv3d_k3_backward(dy, x, w, ctx.pad, ctx.needs_input_grad[0])
    return (dx if ctx.needs_input_grad[0] else None), dw, db, None


conv3d_k3.register_autograd(_backward, setup_context=_setup)


@torch.library.custom_op("nidt::kth_largest", mutates_args=())
def kth_largest(v: torch.Tensor, k: int) -> torch.Tensor:
    from .topk import kth_largest as _k
    return _k(v, k).reshape(())


@kth_largest.register_fake
def _(v, k):
    return v.new_empty(())


@torch.library.custom_op("nidt::weighted_rows_sum", mutates_args=())
def weighted_rows_sum(rows: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if not rows.is_cuda:
        return (w.view(-1, 1).to(rows.dtype) * rows).sum(0)
    if rows.dtype != torch.float32 or w.dtype != torch.float32 or rows.dim() != 2 or w.numel() != rows.shape[0]:
        raise ValueError("nidt::weighted_rows_sum: rows [R,P] fp32, w [R] fp32")
    if rows.stride(1) != 1 or rows.stride(0) % 4 or rows.data_ptr() % 16:
        rows = _padded_copy(rows)
    out = torch.empty(rows.shape[1] + (-rows.shape[1]) % 4, device=rows.device, dtype=torch.float32)
    ext().weighted_rows_sum(rows.data_ptr(), w.contiguous().data_ptr(), rows.shape[0], rows.shape[1], rows.stride(0),
                            0.0, out.data_ptr(), _stream())
    return out[:rows.shape[1]].clone()


def _padded_copy(rows):
    R, P = rows.shape
    ld = P + (-P) % 64
    buf = torch.zeros(R, ld, device=rows.device, dtype=rows.dtype)
    buf[:, :P] = rows
    return buf[:, :P]


@weighted_rows_sum.register_fake
def _(rows, w):
    return rows.new_empty((rows.shape[1],))
