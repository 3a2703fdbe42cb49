"""Per-layer weight-gradient time of the config-5 3D ResNet-50 convs (32 clients x 4 volumes per step) through
GConv3.bwd(need_dx=False) (k_conv_wgrad_dma + k_wgrad_reduce), with effective GB/s (X + dY read once) and TF/s.
Usage: python tools/bench_wgrad3d.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm1x1 import timeit  # noqa: E402


def main():
    from neuroimagedisttraining_amd.engine.resnet3d_hip import GConv3
    dev = torch.device("cuda")
    G, B = 32, 4
    shapes = [  # cin, cout, k, stride, input dims
        (64, 64, 1, 1, (31, 37, 31)), (64, 256, 1, 1, (31, 37, 31)), (256, 64, 1, 1, (31, 37, 31)),
        (64, 64, 3, 1, (31, 37, 31)), (256, 128, 1, 1, (31, 37, 31)), (128, 128, 3, 2, (31, 37, 31)),
        (256, 512, 1, 2, (31, 37, 31)), (128, 512, 1, 1, (16, 19, 16)), (512, 128, 1, 1, (16, 19, 16)),
        (128, 128, 3, 1, (16, 19, 16)), (256, 256, 3, 1, (8, 10, 8)), (512, 512, 3, 1, (4, 5, 4))]
    for cin, cout, k, st, dims in shapes:
        conv = GConv3(0, cout, cin, k, st, (k - 1) // 2)
        P = conv.numel
        theta = torch.randn(G, P, device=dev) * 0.01
        x = torch.randn(G * B, *dims, cin, device=dev).to(torch.bfloat16)
        y = conv.fwd(x, theta, G, train=True)
        dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
        grads = torch.zeros(G, P, device=dev)
        ms = timeit(lambda: conv.bwd(dy, x, theta, grads, G, need_dx=False))
        gb = (x.numel() + dy.numel()) * 2 / 1e9
        tf = 2.0 * dy.numel() * cin * conv.kt / 1e12
        print("cin=%4d cout=%4d k=%d s=%d %-13s wgrad %7.3f ms  %6.0f GB/s  %6.0f TF/s"
              % (cin, cout, k, st, dims, ms, gb / ms * 1e3, tf / ms * 1e3), flush=True)
        del x, y, dy, theta, grads
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
