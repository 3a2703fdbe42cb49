"""Experiment: do lockstep steps of two client cohorts on two HIP streams overlap on the GPU?

Size-skewed federations end each local epoch with many steps of a few large clients (small G: latency-bound
kernels).  Measures T steps of a G_a cohort alone, S steps of a G_b cohort alone, and both replayed as hipGraphs on
two streams at once.  Usage: python tools/exp_streams.py [G_a] [T] [G_b] [S]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    Ga, T, Gb, S = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (1, 76, 63, 18)))
    B = 16
    from neuroimagedisttraining_amd.data.volumes import make_synthetic_abcd
    from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
    from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    dev = torch.device("cuda")
    store = make_synthetic_abcd(256, seed=1, device=dev)
    x8, mom = to_hip_store(store.volumes)
    model = AlexNet3D_Dropout(num_classes=1)
    pl = ParamLayout.from_tensors(list(model.named_parameters()))
    bl = ParamLayout.from_tensors(list(model.named_buffers()))
    net = HipAlexNet3D(pl, bl, dev)

    def cohort(G):
        with torch.no_grad():
            th = padded_rows(G, pl.total, dev)
            th.copy_(pl.flatten_state(dict(model.named_parameters()), dev).unsqueeze(0).expand(G, pl.total))
            bu = padded_rows(G, bl.total, dev)
            bu.copy_(bl.flatten_state(dict(model.named_buffers()), dev).unsqueeze(0).expand(G, bl.total))
        gr = padded_rows(G, pl.total, dev)
        idx = (torch.arange(G * B, device=dev) % x8.shape[0]).int()
        y = store.labels.float().repeat(G * B // store.labels.numel() + 1)[:G * B].contiguous()
        return lambda: net.train_step(th, bu, gr, x8, mom, idx, y, G, B, 0.5, 1)

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    graphs, keep = [], []  # keep: the cohorts' tensors must outlive the graphs (capture empties the cache)
    for G, s in ((Ga, sa), (Gb, sb)):
        fn = cohort(G)
        keep.append(fn)
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        graphs.append(g)
    ga, gb = graphs
    torch.cuda.synchronize()

    def run(parts):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for g, s, n in parts:
            with torch.cuda.stream(s):
                for _ in range(n):
                    g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for _ in range(2):
        ta = run([(ga, sa, T)])
        tb = run([(gb, sb, S)])
        # interleaved enqueue so neither stream waits on the host
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ia = ib = 0
        while ia < T or ib < S:
            if ia < T and (ia * S <= ib * T or ib >= S):
                with torch.cuda.stream(sa):
                    ga.replay()
                ia += 1
            else:
                with torch.cuda.stream(sb):
                    gb.replay()
                ib += 1
        torch.cuda.synchronize()
        tc = (time.perf_counter() - t0) * 1e3
        print("G=%d x %d steps: %.1f ms (%.2f ms/step) | G=%d x %d steps: %.1f ms (%.2f ms/step) | sequential %.1f ms"
              " | two streams %.1f ms" % (Ga, T, ta, ta / T, Gb, S, tb, tb / S, ta + tb, tc), flush=True)


if __name__ == "__main__":
    main()
