"""Bandwidth of the config-5 BatchNorm / residual passes (bnr.hip, gn.hip res_grad) at the layer-1 / layer-2 shapes of
a 32-client x 4-volume lockstep step.  Prints ms and effective GB/s (bytes each kernel must move) per pass.
Usage: python tools/bench_bnr.py"""
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
    G = 32
    for M, C in ((4 * 35557, 64), (4 * 35557, 256), (4 * 4864, 512)):
        t = torch.randn(G, M, C, device=dev).to(torch.bfloat16)
        r = torch.randn(G, M, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(G, M, C, device=dev).to(torch.bfloat16)
        y = torch.empty_like(t)
        P = 4 * C
        theta = torch.randn(G, P, device=dev)
        bufs = torch.zeros(G, 3 * C, device=dev)
        grads = torch.zeros(G, P, device=dev)
        stats = torch.empty(G, C, 2, device=dev)
        coef = torch.empty(G, C, 2, device=dev)
        ws = torch.empty(m.bnr_workspace(G, M, C), device=dev)
        nb = G * M * C * 2 / 1e9

        def stats_fn():
            m.bnr_stats(t.data_ptr(), G, M, C, 1e-5, 0.1, ws.data_ptr(), stats.data_ptr(), bufs.data_ptr(), bufs.stride(0),
                        0, C, -1, st)
        stats_fn()

        def apply_fn():
            m.bnr_apply(t.data_ptr(), r.data_ptr(), stats.data_ptr(), theta.data_ptr(), theta.stride(0), 0, C,
                        y.data_ptr(), G, M, C, 1, st)

        def bwd_fn():
            m.bnr_bwd(t.data_ptr(), dy.data_ptr(), 1, r.data_ptr(), stats.data_ptr(), theta.data_ptr(), theta.stride(0),
                      0, C, grads.data_ptr(), grads.stride(0), ws.data_ptr(), coef.data_ptr(), y.data_ptr(), G, M, C, 0,
                      st)

        def res_fn():
            m.res_grad(y.data_ptr(), t.data_ptr(), 0, dy.data_ptr(), r.data_ptr(), G * M * C, 3, st)

        for name, fn, tensors in (("stats", stats_fn, 1), ("apply+res+relu", apply_fn, 3), ("bwd(partial+apply)", bwd_fn, 7),
                                  ("res_grad", res_fn, 4)):
            ms = timeit(fn)
            print("M=%7d C=%4d %-20s %7.3f ms  %6.0f GB/s (%d tensor passes of %.2f GB)"
                  % (M, C, name, ms, tensors * nb / ms * 1e3, tensors, nb), flush=True)
        del t, r, dy, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
