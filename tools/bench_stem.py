"""Timing of the config-5 stem's pool (k_stem_pool) and unpool / BN backward (k_stem_unpool ...) at 128 volumes of
121x145x121 (32 clients x 4).  Usage: python tools/bench_stem.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm1x1 import timeit  # noqa: E402


def main():
    from neuroimagedisttraining_amd import ops
    m = ops.ext()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    N, B, D, H, W = 128, 4, 121, 145, 121
    OD, OH, OW = (D - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
    QD, QH, QW = (OD - 1) // 2 + 1, (OH - 1) // 2 + 1, (OW - 1) // 2 + 1
    G = N // B
    y = torch.randn(N, OD, OH, OW, 64, device=dev).to(torch.bfloat16)
    scale = torch.rand(G * 64, device=dev) + 0.5
    shift = torch.randn(G * 64, device=dev) * 0.1
    out = torch.empty(N, QD, QH, QW, 64, device=dev, dtype=torch.bfloat16)
    amax = torch.empty(N, QD, QH, QW, 64, device=dev, dtype=torch.uint8)
    ms = timeit(lambda: m.stem_pool(y.data_ptr(), scale.data_ptr(), shift.data_ptr(), N, B, D, H, W, out.data_ptr(),
                                    amax.data_ptr(), st))
    gb = (y.numel() * 2 + out.numel() * 3) / 1e9
    print("stem_pool %.3f ms  %.0f GB/s (y read once, pooled + argmax written)" % (ms, gb / ms * 1e3), flush=True)


if __name__ == "__main__":
    main()
