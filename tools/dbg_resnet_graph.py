"""Debug: capture ResNetHipEngine train_step + local_opt in a CUDA graph and compare with eager."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from neuroimagedisttraining_amd.engine.executor import padded_rows
from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
from neuroimagedisttraining_amd.models import customized_resnet18
dev = torch.device("cuda")
x8, y = synthetic_cifar(64, seed=3)
m = customized_resnet18(class_num=10)
eng = ResNetHipEngine(m, x8, y, dev)
P = eng.players.total
row = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
for G, B in [(4, 8), (1, 1), (2, 3), (1, 4)]:
    th1, g1 = padded_rows(G, P, dev), padded_rows(G, P, dev)
    th1.copy_(row.expand(G, P))
    idx = torch.arange(G * B, dtype=torch.int32, device=dev)
    l1 = eng.train_step(th1, None, g1, idx, G, B, 1.0, 0)
    g2 = padded_rows(G, P, dev)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(gr, capture_error_mode="thread_local"):
            l2 = eng.train_step(th1, None, g2, idx, G, B, 1.0, 0)
        gr.replay()
        torch.cuda.synchronize()
        print(G, B, "captured; losses equal", torch.equal(l1, l2), "grads equal", torch.equal(g1, g2),
              "nan", bool(torch.isnan(g2).any()), float((g1 - g2).abs().max()), flush=True)
    except Exception as e:
        print(G, B, "capture failed:", repr(e)[:300], flush=True)
