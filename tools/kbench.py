"""Per-kernel micro-benchmark at the headline shapes (G clients x B=16, AlexNet3D at 121x145x121).

Runs one full train step to populate every scratch buffer, then re-times each HIP launch of the step in
isolation (median of N reps with HIP events) and prints achieved TFLOP/s against the useful FLOPs of the op.
Usage: python tools/kbench.py [G] [reps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    ts = []
    for _ in range(3):
        fn()
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
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    B = 16
    from neuroimagedisttraining_amd.data.volumes import make_synthetic_abcd
    from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
    from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    dev = torch.device("cuda")
    store = make_synthetic_abcd(min(G * B, 256), seed=1, device=dev)
    x8, mom = to_hip_store(store.volumes)
    model = AlexNet3D_Dropout(num_classes=1)
    pl = ParamLayout.from_tensors(list(model.named_parameters()))
    bl = ParamLayout.from_tensors(list(model.named_buffers()))
    with torch.no_grad():
        theta = padded_rows(G, pl.total, dev)
        theta.copy_(pl.flatten_state(dict(model.named_parameters()), dev).unsqueeze(0).expand(G, pl.total))
        bufs = padded_rows(G, bl.total, dev)
        bufs.copy_(bl.flatten_state(dict(model.named_buffers()), dev).unsqueeze(0).expand(G, bl.total))
    grads = padded_rows(G, pl.total, dev)
    net = HipAlexNet3D(pl, bl, dev)
    idx = (torch.arange(G * B, device=dev) % x8.shape[0]).int()
    y = store.labels.float().repeat((G * B + store.labels.numel() - 1) // store.labels.numel())[:G * B].contiguous()
    step = lambda: net.train_step(theta, bufs, grads, x8, mom, idx, y, G, B, 0.5, 1)  # noqa: E731
    t_step = timeit(step, max(3, reps // 2))
    b = net._cache[(G, B, True)]
    m, st = net.m, torch.cuda.current_stream().cuda_stream
    P = theta.stride(0)
    o = net.o
    p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
    rows = []

    def add(name, fn, flops):
        t = timeit(fn, reps)
        rows.append((name, t, flops / t / 1e9 if flops else 0.0))

    NB = G * B
    add("conv1_fwd_pool", lambda: m.conv1_fwd_pool(p(x8), p(idx), p(b["w1p"]), p(b["s1"]), p(b["t1"]), NB, B, p(b["p1"]),
                                                   p(b["a1"]), st), 2 * 64 * 125 * 57 * 69 * 57 * NB)
    add("conv1_wgrad", lambda: m.conv1_wgrad(p(x8), p(idx), p(b["dp1"]), p(b["p1"]), p(b["a1"]), NB, B, p(b["c1part"]),
                                             p(b["w125"]), p(b["mu"]), p(b["covw"]), p(b["i1"]), p(theta), P,
                                             o["features.1.weight"], p(grads), P, o["features.0.weight"],
                                             o["features.0.bias"], o["features.1.weight"], o["features.1.bias"],
                                             1.0 / 255, 0, st), 2 * 64 * 125 * 19 * 23 * 19 * NB)
    cfgs = [("conv2", "p1", 4, (19, 23, 19), 64, 128, 0), ("conv3", "p2", 8, (5, 7, 5), 128, 192, 1),
            ("conv4", "h3", 11, (5, 7, 5), 192, 192, 1), ("conv5", "h4", 14, (5, 7, 5), 192, 128, 1)]
    outs = {4: "y2", 8: "y3", 11: "y4", 14: "y5"}
    dys = {4: "dy2", 8: "dy3", 11: "dy4", 14: "dy5"}
    dxs = {4: "dp1", 8: "dx3", 11: "dx4", 14: "dx5"}
    for name, xin, ci, sp, cin, cout, pad in cfgs:
        Do = [s + 2 * pad - 2 for s in sp]
        fl = 2.0 * cin * 27 * cout * Do[0] * Do[1] * Do[2] * NB
        # the engine's own launch choice (union-staged k_conv_fwd_tri, split-K or k_conv_fwd_dma)
        add(name + "_fwd", lambda xin=xin, ci=ci, sp=sp, cin=cin, cout=cout, pad=pad: net._conv(
            b, "ksf%d" % ci, b[xin], b["w%dp" % ci], b["bias%d" % ci], b[outs[ci]], b["st%d" % ci], G, B, *sp, cin,
            cout, pad, st), fl)
        add(name + "_dgrad", lambda ci=ci, sp=sp, cin=cin, cout=cout, pad=pad, Do=Do: net._conv(
            b, "ksd%d" % ci, b[dys[ci]], b["w%dt" % ci], None, b[dxs[ci]], None, G, B, *Do, cout, cin, 2 - pad, st), fl)
        if b.get("wslab%d" % ci):  # the engine's kd-slab union wgrad
            add(name + "_wgrad", lambda xin=xin, ci=ci, sp=sp, cin=cin, cout=cout, pad=pad: m.conv3d_wgrad_slab(
                p(b[xin]), p(b[dys[ci]]), p(b["wgpart"]), p(grads), P, o["features.%d.weight" % ci], G, B, *sp, cin,
                cout, pad, b["ns%d" % ci], 1.0, p(b["stab%d" % ci]), st), fl)
            continue
        if b.get("tri%d" % ci):  # the engine's conv2 wgrad (three-tap union staging)
            add(name + "_wgrad", lambda xin=xin, ci=ci, sp=sp, cin=cin, cout=cout, pad=pad: m.conv3d_wgrad_tri(
                p(b[xin]), p(b[dys[ci]]), p(b["wgpart"]), p(grads), P, o["features.%d.weight" % ci], G, B, *sp, cin,
                cout, pad, b["ns%d" % ci], 1.0, p(b["stab%d" % ci]), st), fl)
            continue
        add(name + "_wgrad", lambda xin=xin, ci=ci, sp=sp, cin=cin, cout=cout, pad=pad: m.conv3d_wgrad(
            p(b[xin]), 0, 0, p(b[dys[ci]]), p(b["wgpart"]), p(grads), P, o["features.%d.weight" % ci], G, B, *sp, cin,
            cout, pad, b["ns%d" % ci], 1.0, p(b["pt%d" % ci]), st), fl)
    tot = sum(r[1] for r in rows)
    print("G=%d B=%d  full train step %.3f ms  (sum of timed kernels %.3f ms)" % (G, B, t_step, tot))
    for name, t, tf in rows:
        print("%-16s %9.3f ms  %8.1f TF/s" % (name, t, tf))
    # eval-mode forward at the round's evaluation shape (2G rows: personal + global copies, 36 test samples each)
    if os.environ.get("KBENCH_EVAL", "1") == "1":
        G2, B2 = 2 * G, 36
        th2, bu2 = padded_rows(G2, pl.total, dev), padded_rows(G2, bl.total, dev)
        th2.copy_(theta[:1].expand(G2, -1))
        bu2.copy_(bufs[:1].expand(G2, -1))
        idx2 = (torch.arange(G2 * B2, device=dev) % x8.shape[0]).int()
        t_ev = timeit(lambda: net.eval_logits(th2, bu2, x8, idx2, G2, B2), 3)
        t_tr = timeit(lambda: net.eval_logits(theta, bufs, x8, idx, G, B), 5)
        be = net._cache[(G2, B2, False)]
        t_c1 = timeit(lambda: m.conv1_fwd_pool(p(x8), p(idx2), p(be["w1p"]), p(be["s1"]), p(be["t1"]), G2 * B2, B2,
                                               p(be["p1"]), p(be["a1"]), st), 3)
        bt = net._cache[(G, B, False)]
        t_c1t = timeit(lambda: m.conv1_fwd_pool(p(x8), p(idx), p(bt["w1p"]), p(bt["s1"]), p(bt["t1"]), G * B, B,
                                                p(bt["p1"]), p(bt["a1"]), st), 5)
        print("eval forward %dx%d: %.3f ms (%.2f us/sample; conv1 %.3f ms = %.2f us/sample) | eval forward %dx%d: "
              "%.3f ms (%.2f us/sample; conv1 %.3f ms = %.2f us/sample)"
              % (G2, B2, t_ev, 1e3 * t_ev / (G2 * B2), t_c1, 1e3 * t_c1 / (G2 * B2), G, B, t_tr,
                 1e3 * t_tr / (G * B), t_c1t, 1e3 * t_c1t / (G * B)))


if __name__ == "__main__":
    main()
