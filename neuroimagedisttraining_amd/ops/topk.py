"""Global top-k threshold on the GPU via the HIP radix select (``csrc/kernels/select.hip``)."""
from __future__ import annotations

import torch

from . import ext
from . import stream as _raw_stream


def kth_largest(v: torch.Tensor, k: int) -> torch.Tensor:
    """k-th largest value (1-based) of a non-negative fp32 CUDA tensor, as a 0-d tensor on the same device."""
    if not v.is_cuda:
        return torch.topk(v.flatten(), k, sorted=True).values[-1]
    if v.dtype != torch.float32:
        raise TypeError("kth_largest expects fp32")
    if not (1 <= k <= v.numel()):
        raise ValueError("k out of range")
    m = ext()
    x = v.contiguous().view(-1)
    st = torch.empty(4, dtype=torch.int32, device=v.device)
    hist = torch.empty(256, dtype=torch.int32, device=v.device)
    m.radix_select_kth(x.data_ptr(), x.numel(), int(k), st.data_ptr(), hist.data_ptr(),
                       _raw_stream())
    return st[3:4].view(torch.float32)[0].clone()


def threshold_mask(v: torch.Tensor, k: int) -> torch.Tensor:
    """float mask of ``v >= kth_largest(v, k)`` (ties kept, like the reference's ``>=``)."""
    thr = kth_largest(v, k)
    return (v >= thr).float()
