"""Per-shape timing of the ResNet-18 CIFAR 3x3 stride-1 convs (layers 1-4) on the three forward kernels that can run
them: the kd-slab union kernel (conv2d_fwd_slab, layers 1-2 only), the per-tap LDS-DMA kernel (conv_fwd_g, with its
split-K rule) and the generic implicit-GEMM 2-D kernel (conv2d_any_fwd).  G clients x B images per lockstep step:
G = 10 (SubAvg's sampled clients), 100 (DisPFL's full federation), 100 x 62 (an evaluation chunk).
Usage: python tools/bench_conv2d.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm1x1 import timeit  # noqa: E402


def main():
    from neuroimagedisttraining_amd import ops
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    m = ops.ext()
    dev = torch.device("cuda")
    for G, B in ((10, 16), (100, 16), (100, 62)):
        for H, C in ((32, 64), (16, 128), (8, 256), (4, 512)):
            N = G * B
            x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
            w = (torch.randn(G, C, 9, C, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16)
            y = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
            flop = 2.0 * N * H * H * C * 9 * C
            row = "G=%3d B=%2d %2dx%-2d C=%3d" % (G, B, H, H, C)
            res = {}
            if m.conv2d_fwd_slab_pick(G, B, H, H, C, C):
                res["slab"] = timeit(lambda: R.slab_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, H, H, C, C,
                                                           dev))
                ref = y.clone()
            res["pertap"] = timeit(lambda: R.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, 1, H, H, C, C, 9,
                                                      1, 1, 0, dev))
            ref = y.clone()
            if m.conv2d_fwd_slab_bd_ok(B, H, H, C, C):  # samples as depth planes (tools: always timed when eligible)
                tab = torch.empty(m.conv2d_fwd_slab_bd_table_size(B, H, H, C, C), device=dev, dtype=torch.int32)
                m.conv2d_fwd_slab_bd_table(tab.data_ptr(), B, H, H, C, C, ops.stream())
                y.zero_()
                res["slab_bd"] = timeit(lambda: m.conv2d_fwd_slab_bd(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, H, H,
                                                                     C, C, tab.data_ptr(), ops.stream()))
                row += "  [bd vs pertap rel %.1e]" % float((y.float() - ref.float()).norm() / ref.float().norm())
            res["any"] = timeit(lambda: m.conv2d_any_fwd(x.data_ptr(), w.data_ptr(), 0, y.data_ptr(), G, B, H, H, C, C,
                                                         C, 3, 1, ops.stream()))
            err = float((y.float() - ref.float()).norm() / ref.float().norm())
            for k, t in res.items():
                row += "  %s %.3f ms %.0f TF/s" % (k, t, flop / t / 1e9)
            print(row + "  (any vs pertap rel %.1e)" % err, flush=True)
            del x, w, y, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
