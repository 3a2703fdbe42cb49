"""Timing of the register-resident GroupNorm kernels (gn.hip) at the CIFAR ResNet-18-GN shapes of a 100-client DisPFL
step (1600 samples): forward (with / without the residual) and backward per layer map, with the effective HBM bytes/s
(activation read + write, residual / dy / mask reads).  Usage: python tools/bench_gn.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm1x1 import timeit  # noqa: E402


def main():
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupNormG
    dev = torch.device("cuda")
    G, B = 100, 16
    N = G * B
    for hw, C in ((32, 64), (16, 128), (8, 256), (4, 512)):
        theta = torch.randn(G, 2 * C + 64, device=dev)
        gn = GroupNormG(0, C, C, hip=True)
        t = torch.randn(N, hw, hw, C, device=dev).to(torch.bfloat16)
        r = torch.randn(N, hw, hw, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, hw, hw, C, device=dev).to(torch.bfloat16)
        grads = torch.zeros_like(theta)
        nb = t.numel() * 2
        y, st = gn.fwd(t, theta, G, relu=True)
        tf = timeit(lambda: gn.fwd(t, theta, G, relu=True))
        tr = timeit(lambda: gn.fwd(t, theta, G, res=r, relu=True))
        tb = timeit(lambda: gn.bwd(dy, y, t, st, theta, grads, G))
        print("%2dx%-2d C=%3d  fwd %.3f ms (%.2f TB/s)  fwd+res %.3f ms (%.2f TB/s)  bwd %.3f ms (%.2f TB/s)"
              % (hw, hw, C, tf, 2 * nb / tf / 1e9, tr, 3 * nb / tr / 1e9, tb, 4 * nb / tb / 1e9), flush=True)


if __name__ == "__main__":
    main()
