"""Per-shape timing of the 1x1x1 stride-1 convs of config 5 (3D ResNet-50, 32 clients x 4 volumes per lockstep step):
the streaming GEMM kernel (gemm1x1.hip) vs the general LDS-DMA conv kernel (conv_fwd_g with one tap).  Prints ms,
effective HBM GB/s (X read once + Y written once) and TF/s per shape.  Usage: python tools/bench_gemm1x1.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from neuroimagedisttraining_amd import ops
    m = ops.ext()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    G, B = 32, 4
    # (K, N, spatial): layer 1 at 31x37x31, layer 2 at 16x19x16, layer 3 at 8x10x8
    shapes = [(64, 64, (31, 37, 31)), (64, 256, (31, 37, 31)), (256, 64, (31, 37, 31)), (256, 128, (31, 37, 31)),
              (128, 512, (16, 19, 16)), (512, 128, (16, 19, 16)), (128, 256, (16, 19, 16)),
              (256, 1024, (8, 10, 8)), (512, 256, (8, 10, 8))]
    for K, N, (D, H, W) in shapes:
        Mg = B * D * H * W
        x = torch.randn(G * B, D, H, W, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(G, N, 1, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        y = torch.empty(G * B, D, H, W, N, device=dev, dtype=torch.bfloat16)
        y2 = torch.empty_like(y)
        t_old = timeit(lambda: m.conv_fwd_g(x.data_ptr(), w.data_ptr(), y2.data_ptr(), G, B, D, H, W, K, N, 1, 1, 0, 0,
                                            st))
        line = "K=%4d N=%4d Mg=%6d  conv_fwd_g %7.3f ms" % (K, N, Mg, t_old)
        if m.gemm1x1_ok(K, N):
            t_new = timeit(lambda: m.gemm1x1_g(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, Mg, K, N, 0, st))
            gb = G * Mg * (K + N) * 2 / 1e9
            tf = 2.0 * G * Mg * K * N / 1e12
            err = float((y.float() - y2.float()).norm() / y2.float().norm())
            line += " | gemm1x1 %7.3f ms  %6.0f GB/s  %6.0f TF/s  (x%.2f, rel diff %.1e)" % (
                t_new, gb / t_new * 1e3, tf / t_new * 1e3, t_old / t_new, err)
        print(line, flush=True)
        del x, y, y2, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
