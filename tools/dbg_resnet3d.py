"""Debug: per-parameter gradient agreement of the client-batched ResNet3D step vs per-client autograd."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from torch.func import functional_call
from neuroimagedisttraining_amd.engine.executor import padded_rows
from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
from neuroimagedisttraining_amd.models.resnet3d import resnet3d_50
dev = torch.device("cuda")
torch.manual_seed(0)
G, B = 2, 2
vol = torch.randint(0, 256, (G * B, 40, 48, 40), dtype=torch.uint8, device=dev)
lab = torch.tensor([0.0, 1.0, 1.0, 0.0], device=dev)
m = resnet3d_50(num_classes=1)
eng = ResNet3DHipEngine(m, vol, lab, dev)
L, Lb = eng.players, eng.blayers
flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
bflat = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()]).to(dev)
th, gr = padded_rows(G, L.total, dev), padded_rows(G, L.total, dev)
bu = padded_rows(G, Lb.total, dev)
th.copy_(flat.expand(G, -1)); bu.copy_(bflat.expand(G, -1))
idx = torch.arange(G * B, dtype=torch.int32, device=dev)
losses = eng.train_step(th, bu, gr, idx, G, B, 1.0, 0)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_resnet3d import _bf16_faithful
mref = _bf16_faithful(resnet3d_50(num_classes=1).to(dev)); mref.train()
conv_names = {n + ".weight" for n, mod in mref.named_modules() if isinstance(mod, torch.nn.Conv3d)}
g = 0
row = flat.clone().requires_grad_(True)
pv = {n: (row[o:o + L.numel(i)].view(L.shapes[i]).to(torch.bfloat16).float() if n in conv_names else row[o:o + L.numel(i)].view(L.shapes[i])) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
bv = {n: bflat[o:o + Lb.numel(i)].view(Lb.shapes[i]).clone().to(Lb.dtypes[i]) for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets))}
x = (vol[:B].float().unsqueeze(1) / 255.0).to(torch.bfloat16).float()
out = functional_call(mref, {**pv, **bv}, (x,))
loss = F.binary_cross_entropy_with_logits(out.view(-1), lab[:B]); loss.backward()
print("loss", float(loss), float(losses[0]))
for i, (n, o) in enumerate(zip(L.names, L.offsets)):
    a = gr[0, o:o + L.numel(i)]; b = row.grad[o:o + L.numel(i)]
    cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
    print("%-40s cos %.4f  |a| %.3e |b| %.3e" % (n, cos, float(a.norm()), float(b.norm())))
