"""Per-layer timings of the client-batched ResNet-18-GN (CIFAR) convolutions and GroupNorm kernels.

For every distinct conv shape of ``customized_resnet18`` at G clients x B=16 images: forward, data-gradient and
weight-gradient time (median of N reps, HIP events) and achieved TFLOP/s on the useful FLOPs; then one whole
lockstep train step.  Usage: python tools/kbench_resnet.py [G] [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupedConv, GroupNormG, ResNetHipEngine, synthetic_cifar
    from neuroimagedisttraining_amd.models import customized_resnet18
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    B = 16
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = [(3, 64, 3, 1, 1, 32), (64, 64, 3, 1, 1, 32), (64, 128, 3, 2, 1, 32), (64, 128, 1, 2, 0, 32),
              (128, 128, 3, 1, 1, 16), (128, 256, 3, 2, 1, 16), (256, 256, 3, 1, 1, 8), (256, 512, 3, 2, 1, 8),
              (512, 512, 3, 1, 1, 4)]
    print("G=%d B=%d" % (G, B))
    for cin, cout, k, st, pad, hw in shapes:
        conv = GroupedConv(0, cout, cin, k, st, pad, hip=True)
        P = conv.numel
        theta = padded_rows(G, P, dev)
        theta.copy_(torch.randn(G, P, device=dev) * 0.05)
        grads = padded_rows(G, P, dev)
        x = torch.randn(G * B, hw, hw, conv.cin_p, device=dev).to(torch.bfloat16)
        y = conv.fwd(x, theta, G, train=True)
        dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
        ho = y.shape[1]
        flops = 2.0 * G * B * ho * ho * cout * cin * k * k
        tf = timeit(lambda: conv.fwd(x, theta, G), reps)
        tb = timeit(lambda: (conv.fwd(x, theta, G, train=True), conv.bwd(dy, x, theta, grads, G, cin % 64 == 0)),
                    reps) - tf
        print("conv %4d->%-4d k%d s%d %2dx%-2d  fwd %7.3f ms %7.1f TF/s | bwd(dgrad+wgrad) %7.3f ms %7.1f TF/s"
              % (cin, cout, k, st, hw, hw, tf, flops / tf / 1e9, tb, (2 if cin % 64 == 0 else 1) * flops / tb / 1e9))
    for C, hw in [(64, 32), (128, 16), (256, 8), (512, 4)]:
        gn = GroupNormG(0, C, C, hip=True)
        theta = torch.ones(G, 2 * C + 64, device=dev)
        grads = torch.zeros_like(theta)
        t = torch.randn(G * B, hw, hw, C, device=dev).to(torch.bfloat16)
        y, stt = gn.fwd(t, theta, G, relu=True)
        dy = torch.randn(y.shape, device=dev)
        tf = timeit(lambda: gn.fwd(t, theta, G, relu=True), reps)
        tb = timeit(lambda: gn.bwd(dy, y, t, stt, theta, grads, G), reps)
        mb = t.numel() * 2 / 1e6
        print("groupnorm C=%-3d %2dx%-2d  fwd %7.3f ms (%6.0f GB/s) | bwd %7.3f ms" % (C, hw, hw, tf, 2 * mb / tf, tb))
    m = customized_resnet18(class_num=10)
    x8, yl = synthetic_cifar(G * B, seed=1)
    eng = ResNetHipEngine(m, x8, yl, dev)
    P = eng.players.total
    th, gr = padded_rows(G, P, dev), padded_rows(G, P, dev)
    th.copy_(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev).expand(G, P))
    idx = torch.arange(G * B, dtype=torch.int32, device=dev)
    ts = timeit(lambda: eng.train_step(th, None, gr, idx, G, B, 1.0, 0), reps)
    fl = 3 * 2 * 0.556e9 * G * B
    print("full lockstep train step (eager, G=%d): %.3f ms  (%.0f TF/s on ~%.2f TFLOP)" % (G, ts, fl / ts / 1e9,
                                                                                          fl / 1e12))


if __name__ == "__main__":
    main()
