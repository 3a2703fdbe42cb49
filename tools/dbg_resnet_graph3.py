"""Debug: poison the caching allocator's free memory between replays; report which gradients go NaN."""
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
L = eng.players
P = L.total
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
free, tot = torch.cuda.mem_get_info()
junk = [torch.full((64 << 20,), float("nan"), device=dev) for _ in range(8)]
del junk
torch.cuda.synchronize()
g.replay(); torch.cuda.synchronize()
print("after poison equal", torch.equal(gr, gr2), flush=True)
for i, (n, o) in enumerate(zip(L.names, L.offsets)):
    seg = gr2[:, o:o + L.numel(i)]
    if not torch.isfinite(seg).all() or not torch.equal(seg, gr[:, o:o + L.numel(i)]):
        print("  differs:", n, "nan" if torch.isnan(seg).any() else "", float((seg - gr[:, o:o + L.numel(i)]).abs().nan_to_num(9).max()))
