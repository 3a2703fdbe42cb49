"""Debug: replay a captured ResNet step after unrelated eager work (eval / other shapes) and compare with eager."""
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
G, B = 4, 8
th, gr = padded_rows(G, P, dev), padded_rows(G, P, dev)
th.copy_(row.expand(G, P))
idx = torch.arange(G * B, dtype=torch.int32, device=dev)
eng.train_step(th, None, gr, idx, G, B, 1.0, 0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
gr2 = padded_rows(G, P, dev)
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    l2 = eng.train_step(th, None, gr2, idx, G, B, 1.0, 0)
g.replay(); torch.cuda.synchronize()
print("replay1 equal", torch.equal(gr, gr2), flush=True)
# unrelated eager work: eval of other shapes, a train step with another G
for k in range(3):
    th1 = padded_rows(1, P, dev); th1.copy_(row[None]); gg = padded_rows(1, P, dev)
    eng.train_step(th1, None, gg, idx[:3], 1, 3, 1.0, 0)
    eng.eval_logits(th, None, idx, G, B)
    torch.cuda.synchronize()
    g.replay(); torch.cuda.synchronize()
    print("after eager work", k, "equal", torch.equal(gr, gr2), "nan", bool(torch.isnan(gr2).any()),
          float((gr - gr2).abs().nan_to_num(9).max()), flush=True)
# second graph of another shape, then replay the first
g2 = torch.cuda.CUDAGraph()
th1 = padded_rows(2, P, dev); th1.copy_(row.expand(2, P)); gg = padded_rows(2, P, dev)
eng.train_step(th1, None, gg, idx[:6], 2, 3, 1.0, 0)
with torch.cuda.graph(g2, capture_error_mode="thread_local"):
    eng.train_step(th1, None, gg, idx[:6], 2, 3, 1.0, 0)
g2.replay()
g.replay(); torch.cuda.synchronize()
print("after 2nd graph equal", torch.equal(gr, gr2), "nan", bool(torch.isnan(gr2).any()), flush=True)
